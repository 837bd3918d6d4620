#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
SKIP_TESTS=1 AB_WLS="${AB_WLS}" VARIANTS="${VARIANTS}" bash scripts/gpu_iter3.sh || exit 1
bash scripts/gpu_rehearse_multi.sh
