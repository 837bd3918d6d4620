#!/bin/bash
# Round 4: self-contained mode-3 decode descriptors (one round trip for the chunk's geometry):
# parity, then A/B against the previous HEAD's library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4m gpurun_out/ab
rm -f gpurun_out/ab/summary.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_arctopk.py tests/test_gpu_multirank.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r4m/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4m/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/r4m/tests.log | head -20; exit $rc; }
AB_LIBS=prev BENCH_ARGS="--workload resnet18_conv --steps 30" VARIANTS="product" bash scripts/gpu_ab_lib.sh || exit 1
AB_LIBS=prev BENCH_ARGS="--workload resnet18_ddp --steps 30" VARIANTS="product" bash scripts/gpu_ab_lib.sh || exit 1
AB_LIBS=prev BENCH_ARGS="--workload resnet50_mixed --steps 30" VARIANTS="product" bash scripts/gpu_ab_lib.sh || exit 1
AB_LIBS=prev BENCH_ARGS="--workload headline --steps 30" VARIANTS="product" bash scripts/gpu_ab_lib.sh || exit 1
