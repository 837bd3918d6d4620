#!/bin/bash
# Short-row decode A/B + kernel traces of the weak workloads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SKIP_TESTS=1 AB_WLS="--workload,resnet18_conv --workload,resnet50_mixed --workload,resnet18_ddp" VARIANTS="base quad0" bash scripts/gpu_iter3.sh || exit 1
KSEQ_BACK=7 TRACES="r18ddp --workload resnet18_ddp
llama --workload llama_embed
noef --ef noef
bf16 --dtype bf16
r18conv --workload resnet18_conv" bash scripts/gpu_traces.sh
