#!/bin/bash
# GPU parity suite only (pass extra pytest args, e.g. a -k filter, in PYTEST_ARGS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -15
tail -3 gpurun_out/pytest_gpu.log
exit $rc
