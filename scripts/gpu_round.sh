#!/bin/bash
# Full GPU pass: parity tests, then every workload through bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 240 -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc -- stopping"; tail -60 gpurun_out/pytest_gpu.log; exit $rc; fi
bash scripts/gpu_workloads.sh
if [ -n "${ENC_PROBE}" ]; then
  timeout -k 10 300 python scripts/enc_probe.py > gpurun_out/enc_probe.log 2>&1 || { echo "enc_probe failed"; tail -20 gpurun_out/enc_probe.log; exit 1; }
  grep -v amdgpu gpurun_out/enc_probe.log
fi
