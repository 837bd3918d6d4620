#!/bin/bash
# Round-3 iteration: GPU parity suite at HEAD, then A/B of library variants on the weak workloads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "${SKIP_TESTS}" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc -- stopping"; grep -E "Error|FAIL|assert" gpurun_out/pytest_gpu.log | head -40; exit $rc; fi
for wl in ${AB_WLS}; do
  BENCH_ARGS="${wl//,/ }" VARIANTS="${VARIANTS}" bash scripts/gpu_ab_lib.sh || exit 1
done
