#!/bin/bash
# rocprofv3 kernel traces of the main workloads (no markers in the timed region) and the
# per-call phase table built from them (scripts/trace_table.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
dirs=""
while read -r tag args; do
  [ -z "$tag" ] && continue
  BENCH_ARGS="$args" bash scripts/trace_wl.sh "wl_$tag" > gpurun_out/t_wl_$tag.txt 2>&1 || { echo "trace $tag failed"; tail -5 gpurun_out/t_wl_$tag.txt; exit 1; }
  dirs="$dirs gpurun_out/trace_wl_$tag"
  echo "$tag done"
done <<LIST
ef14 --workload headline --ef ef14
ef21 --workload headline --ef ef21
noef --workload headline --ef noef
bf16 --workload headline --ef ef14 --dtype bf16
fx --workload headline --ef ef14 --force-exchange
llama --workload llama_embed --ef ef14
roberta --workload roberta_embed --ef ef14
r18c --workload resnet18_conv --ef ef14
r50 --workload resnet50_mixed --ef ef14
layer --workload llama_layer_mixed --ef ef14
r18 --workload resnet18_ddp --ef ef14
r18fx --workload resnet18_ddp --ef ef14 --force-exchange
${EXTRA_WL}
LIST
python3 scripts/trace_table.py $dirs | tee gpurun_out/trace_table.txt
