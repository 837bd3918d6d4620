#!/bin/bash
# rocprofv3 evidence for bench.py: kernel trace + stats, then separate PMC passes for
# FETCH_SIZE and WRITE_SIZE (TCC counters cannot share one pass).  Usage: profile.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
# the step path only (no forced-exchange / emulated-wire sub-runs): the launches bench.py's roofline
# times, so the rocprofv3 average and the PMC bytes describe the same kernel launches
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --no-forced-exchange --wire-busbw ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/bench_trace.log; exit 1; }
tail -1 $OUT/bench_trace.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/bench_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/bench_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/bench_write.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/bench_write.log; exit 1; }
find $OUT -name "*.csv" | head -20
python3 scripts/summarize_prof.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
