#!/bin/bash
# A/B of runtime tuning switches through bench.py: CONFIGS holds ';'-separated env sets.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/envab
IFS=';' read -ra SETS <<< "${CONFIGS}"
for rep in 1 2; do
  i=0
  for cfg in "${SETS[@]}"; do
    i=$((i+1))
    for ef in ${EFS:-ef14}; do
      log=gpurun_out/envab/c$i.$ef.$rep.log
      env $cfg timeout -k 10 200 python bench.py --ef $ef --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > $log 2>&1 || { echo "bench [$cfg] failed"; tail -20 $log; exit 1; }
      python - "[$cfg] $ef" $log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["phase_ms"]
print(f"{sys.argv[1]:44s} {d['value']:8.1f} GB/s  ms/bucket {d['ms_per_bucket']:.4f}  " +
      "  ".join(f"{k[:6]} {v*1e3:6.1f}" for k, v in ph.items() if "allreduce" not in k))
PY
    done
  done
done
