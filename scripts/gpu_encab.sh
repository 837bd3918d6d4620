#!/bin/bash
# Encode A/B: traces of the weak workloads, then library variants (lib/var) on each workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
KSEQ_BACK=7 TRACES="r18ddp --workload resnet18_ddp
llama --workload llama_embed
roberta --workload roberta_embed
noef --ef noef
bf16 --dtype bf16" bash scripts/gpu_traces.sh || exit 1
for wl in "--ef noef" "--workload llama_embed" "--dtype bf16" "--ef ef14"; do
  BENCH_ARGS="$wl" VARIANTS="${VARIANTS}" bash scripts/gpu_ab_lib.sh || exit 1
done
