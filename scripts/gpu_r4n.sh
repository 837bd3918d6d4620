#!/bin/bash
# Round 4: persistent mode-3 decode (next chunk's loads in flight during this chunk's stores):
# parity on the conv stack (all chunks mode 3), then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4n gpurun_out/ab
rm -f gpurun_out/ab/summary.txt
for v in p1024 p2048; do
  ARCTOPK_LIB=allreducetopk_amd/lib/var/libarctopk_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_arctopk.py -m gpu -q -k "conv3x3 or resnet18 or end_to_end or golden or bf16 or phases" --timeout 120 --timeout-method thread > gpurun_out/r4n/${v}_tests.log 2>&1
  rc=$?; tail -1 gpurun_out/r4n/${v}_tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/r4n/${v}_tests.log | head; exit $rc; }
done
BENCH_ARGS="--workload resnet18_conv --steps 30" VARIANTS="p1024 p2048" bash scripts/gpu_ab_lib.sh || exit 1
BENCH_ARGS="--workload resnet18_conv --ef ef21 --steps 30" VARIANTS="p1024 p2048" bash scripts/gpu_ab_lib.sh || exit 1
