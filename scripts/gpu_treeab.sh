#!/bin/bash
# Same-box A/B of two source trees (ab_old = an earlier commit's worktree, . = current).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/treeab
for rep in 1 2; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS}) > gpurun_out/treeab/$rep.$(basename $(realpath $tree)).log 2>&1 || { echo "bench in $tree failed"; exit 1; }
    tail -1 gpurun_out/treeab/$rep.$(basename $(realpath $tree)).log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tree', d['value'], d['ms_per_step'], {k: round(v*1e3,1) for k,v in d.get('phase_ms',{}).items()})"
  done
done
