#!/bin/bash
# A/B: phase timing with device-scope vs torch (system-scope) events; V-ready event scope.
# Then a rocprof kernel trace of the default bench for the encode average and idle gaps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/evab
O=gpurun_out/evab
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
B="python bench.py --steps 50 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 $B > $O/dev.log 2>&1 || { tail -20 $O/dev.log; exit 1; }
timeout -k 10 200 $B --system-events > $O/sys.log 2>&1 || { tail -20 $O/sys.log; exit 1; }
ARCTOPK_V_READY_SCOPE=device timeout -k 10 200 $B > $O/vdev.log 2>&1 || { tail -20 $O/vdev.log; exit 1; }
for f in dev sys vdev; do
  python - $O/$f.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(sys.argv[1], "value", d["value"], "enc_us", r["avg_launch_us"], "frac", r["frac"], "phases", d["phase_ms"])
PY
done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
tail -1 $O/prof.log
S=$(find $O/prof -name "*kernel_stats.csv" | head -1); T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
head -8 "$S"
python scripts/gaps.py "$T"
