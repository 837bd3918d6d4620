#!/bin/bash
# rocprofv3 kernel trace of one bench workload (no PMC): per-kernel averages + one call's launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-wl}
OUT=gpurun_out/trace_${TAG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-phase-events --no-forced-exchange ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { echo "trace failed"; tail -20 $OUT/bench.log; exit 1; }
python3 scripts/kseq.py $(find $OUT -name "*kernel_trace.csv" | head -1)
