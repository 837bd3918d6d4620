#!/bin/bash
# bench.py on every workload (EF14) and on the headline bucket in all EF modes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/wl
: > gpurun_out/wl/all.jsonl
for spec in "headline ef14" "headline ef21" "headline noef" "llama_embed ef14" "roberta_embed ef14" \
            "resnet18_conv ef14" "resnet50_mixed ef14" "llama_layer_mixed ef14" ${EXTRA_WL}; do
  set -- $spec
  timeout -k 10 240 python bench.py --workload $1 --ef $2 --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/wl/$1_$2.log 2>&1 || { echo "bench $1 $2 failed"; tail -20 gpurun_out/wl/$1_$2.log; exit 1; }
  tail -1 gpurun_out/wl/$1_$2.log >> gpurun_out/wl/all.jsonl
  echo "$1 $2 done"
done
