#!/bin/bash
# Bench lines on one GPU box: one `bench.py` run per line of the list file $1 (arguments of
# one run per line; blank lines and lines starting with # skipped), each under its own time
# limit, JSON lines collected into gpurun_out/$OUT/wl.jsonl and summarised by wl_table.py.
#   OUT=r5a bash scripts/gpu_bench.sh scripts/lists/baseline.txt
# Stops at the first failing run (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-bench}
mkdir -p "$OUT"
: > "$OUT/wl.jsonl"
i=0
while read -r args; do
  case "$args" in ''|'#'*) continue ;; esac
  i=$((i+1))
  timeout -k 10 ${RUN_LIMIT:-240} python bench.py $args > "$OUT/w$i.log" 2>&1 || {
    echo "bench [$args] failed rc=$?"; tail -20 "$OUT/w$i.log"; exit 1; }
  tail -1 "$OUT/w$i.log" >> "$OUT/wl.jsonl"
  echo "[$args] done"
done < "$1"
python scripts/wl_table.py "$OUT/wl.jsonl" > "$OUT/workloads_table.txt" && cat "$OUT/workloads_table.txt"
