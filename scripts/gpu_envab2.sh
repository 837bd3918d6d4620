#!/bin/bash
# env-knob A/B through bench.py (two reps each, interleaved): $KNOBS = space-separated VAR=val
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/envab
for rep in 1 2; do
  for k in X=0 $KNOBS; do
    env $k timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/envab/$k.$rep.log 2>&1 || { echo "$k failed"; tail -20 gpurun_out/envab/$k.$rep.log; exit 1; }
    python3 - "$k" gpurun_out/envab/$k.$rep.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
ph = d["phase_ms"]
print(f"{sys.argv[1]:32s} value {d['value']:8.1f}  " + "  ".join(f"{k} {v*1e3:6.1f}" for k, v in ph.items()), flush=True)
PY
  done
done
