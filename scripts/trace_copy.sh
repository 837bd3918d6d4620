#!/bin/bash
# Kernel + memory-copy + HIP API trace (no PMC) of a short headline bench: where the
# projection H2D copies sit relative to the kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/trace_copy
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-phase-events ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { echo "trace failed"; tail -20 $OUT/bench.log; exit 1; }
ls $OUT
