#!/bin/bash
# Round 4: the new GPU tests first (all reported), then the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4t
timeout -k 10 400 python -u -m pytest tests/test_gpu_exchange_failures.py tests/test_gpu_sparse.py tests/test_gpu_arctopk.py -m gpu -v -k "exchange_failures or randk or rccl or wire or direct or aborted or window" --timeout 120 --timeout-method thread > gpurun_out/r4t/new.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r4t/new.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4t/pytest_gpu.log 2>&1
rc2=$?
grep -E "FAILED|ERROR" gpurun_out/r4t/pytest_gpu.log | tail -15
tail -3 gpurun_out/r4t/pytest_gpu.log
exit $(( rc || rc2 ))
