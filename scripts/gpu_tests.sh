#!/bin/bash
# GPU tests on one box: `bash scripts/gpu_tests.sh [pytest selection...]` (default: the whole
# -m gpu suite), log in gpurun_out/$OUT/pytest_gpu.log; stops the call on failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-tests}
mkdir -p "$OUT"
[ $# -eq 0 ] && set -- tests
timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest "$@" -m gpu -x -v --timeout 240 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then
  echo "pytest rc=$rc"; grep -E "Error|FAIL|assert" "$OUT/pytest_gpu.log" | head -40; exit $rc
fi
