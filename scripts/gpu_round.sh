#!/bin/bash
# Full GPU pass: parity tests, the default bench line (with CPU baseline), every workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc -- stopping"; grep -E "Error|FAIL|assert" gpurun_out/pytest_gpu.log | head -40; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
bash scripts/gpu_workloads.sh
