#!/bin/bash
# Round 4 A/B (interleaved, two repetitions): short-row decode mode 3 vs mode 2, the
# first-digit window on / off, the fused select write at wider spans.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -f gpurun_out/ab/summary.txt
BENCH_ARGS="--workload resnet18_conv --steps 30" VARIANTS="dec2 nowin span2" bash scripts/gpu_ab_lib.sh || exit 1
BENCH_ARGS="--workload resnet50_mixed --steps 30" VARIANTS="nowin span2big span4big" bash scripts/gpu_ab_lib.sh || exit 1
BENCH_ARGS="--workload resnet18_ddp --steps 30" VARIANTS="nowin span2" bash scripts/gpu_ab_lib.sh || exit 1
