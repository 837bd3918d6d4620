#!/bin/bash
# A/B of library variants on one box: bench.py (args in BENCH_ARGS) with each lib, interleaved.
# Summary lines go to stdout and gpurun_out/ab/summary.txt (appended, tagged by BENCH_ARGS).
# FORCED=1 also times the forced-exchange (N > 1 code path) leg of each run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
TAG=$(echo "${BENCH_ARGS}" | tr -c 'a-zA-Z0-9_' '_' | sed 's/__*/_/g')
FX="--no-forced-exchange"
[ "${FORCED:-0}" = 1 ] && FX=""
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${AB_LIBS:-product} ${VARIANTS}; do
    if [ "$lib" = product ]; then L=""; else L="allreducetopk_amd/lib/var/libarctopk_$lib.so"; fi
    LOG=gpurun_out/ab/${lib}${TAG}.log
    ARCTOPK_LIB=$L timeout -k 10 200 python bench.py --steps ${STEPS:-50} --no-cpu-baseline $FX --wire-busbw ${BENCH_ARGS} > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
    tail -1 $LOG | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms']; fx=d.get('forced_exchange') or {}; r=d.get('roofline') or {}; print('${BENCH_ARGS}', '$lib', d['config']['hook_path'], d['value'], 'fx', fx.get('value'), round(r.get('avg_launch_us') or 0,1), round((r.get('hook') or {}).get('device_us') or 0,1), 'frac', r.get('frac'), {k: round(v*1e3,1) for k,v in p.items()})" | tee -a gpurun_out/ab/summary.txt
  done
done
