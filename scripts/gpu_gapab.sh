#!/bin/bash
# GPU parity tests, then kernel traces of the default bench (and $VARIANTS as name:ENV=val) with idle-gap analysis.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/gapab
mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/$name -o run -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/$name.log 2>&1 || { echo "$name failed"; tail -20 $O/$name.log; return 1; }
  echo "== $name: $(grep -o '"value": [0-9.]*' $O/$name.log) $(grep -o '"avg_launch_us": [0-9.]*' $O/$name.log)"
  python3 scripts/gaps.py $(find $O/$name -name "*kernel_trace.csv" | head -1)
}
run base ARCTOPK_X=0 || exit 1
for v in $VARIANTS; do run ${v%%:*} ${v#*:} || exit 1; done
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_plain.log 2>&1 || { tail -20 $O/bench_plain.log; exit 1; }
tail -1 $O/bench_plain.log
