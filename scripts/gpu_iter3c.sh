#!/bin/bash
# Encode A/B: GPU parity of the encode changes, small-bucket tiles, then encode variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_arctopk.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
SKIP_TESTS=1 AB_WLS="--workload,resnet18_ddp --workload,resnet50_mixed --workload,headline" VARIANTS="base mt2k mt4k" bash scripts/gpu_iter3.sh || exit 1
SKIP_TESTS=1 AB_LIBS=" " AB_WLS="--ef,noef --workload,llama_embed --dtype,bf16" VARIANTS="base gonly8 tb1024 tb4096 noil pkfma bf16u8" bash scripts/gpu_iter3.sh
