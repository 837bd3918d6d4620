#!/bin/bash
# rocprofv3 kernel traces (no PMC) of several workloads: per-kernel averages + one call's launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
while read -r tag args; do
  [ -z "$tag" ] && continue
  BENCH_ARGS="$args" bash scripts/trace_wl.sh $tag > gpurun_out/t_$tag.txt 2>&1 || { echo "trace $tag failed"; tail -20 gpurun_out/t_$tag.txt; exit 1; }
  echo "== $tag"; head -14 gpurun_out/t_$tag.txt
done <<LIST
${TRACES:-r18ddp --workload resnet18_ddp}
LIST
