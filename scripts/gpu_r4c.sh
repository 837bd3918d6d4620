#!/bin/bash
# Round 4: GPU tests (the select ones first, then the suite), then the A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4t
timeout -k 10 300 python -u -m pytest tests/test_gpu_arctopk.py -m gpu -v -k "window_across_calls or end_to_end" --timeout 120 --timeout-method thread > gpurun_out/r4t/sel.log 2>&1
rc=$?; grep -E "PASSED|FAILED|distinct rows" gpurun_out/r4t/sel.log | head -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4t/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/r4t/pytest_gpu.log | tail -8; tail -2 gpurun_out/r4t/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r4ab.sh
