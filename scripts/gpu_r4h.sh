#!/bin/bash
# Round 4: mode-3 decode chunk size / store variants (parity of the 8192-element chunk, then A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4h gpurun_out/ab
rm -f gpurun_out/ab/summary.txt
for v in c8192 c2048; do
  ARCTOPK_LIB=allreducetopk_amd/lib/var/libarctopk_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_arctopk.py -m gpu -q -k "conv3x3 or resnet18 or resnet50 or end_to_end or golden or bf16" --timeout 120 --timeout-method thread > gpurun_out/r4h/${v}_tests.log 2>&1
  rc=$?; tail -1 gpurun_out/r4h/${v}_tests.log; [ $rc -eq 0 ] || exit $rc
done
BENCH_ARGS="--workload resnet18_conv --steps 30" VARIANTS="c2048 c8192 c8192v ntoff" bash scripts/gpu_ab_lib.sh || exit 1
BENCH_ARGS="--workload resnet50_mixed --steps 30" VARIANTS="c2048 c8192 ntoff" bash scripts/gpu_ab_lib.sh || exit 1
BENCH_ARGS="--workload resnet18_ddp --steps 30" VARIANTS="c2048 c8192" bash scripts/gpu_ab_lib.sh || exit 1
echo done
