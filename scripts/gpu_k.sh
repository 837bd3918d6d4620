#!/bin/bash
# GPU tests selected by a -k expression: K="expr" bash scripts/gpu_k.sh (prints stdout: -s)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_k.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|flips" gpurun_out/pytest_k.log | tail -40
tail -3 gpurun_out/pytest_k.log
exit $rc
