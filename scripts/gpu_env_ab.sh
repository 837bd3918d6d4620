#!/bin/bash
# A/B of environment settings on one box (ENVS: space-separated VAR=value[,VAR=value] sets, "-"
# for none): bench.py $BENCH_ARGS under each, interleaved, REPS times.  FORCED=1 adds the forced-
# exchange leg.  Lines go to stdout and gpurun_out/ab/env_summary.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
FX="--no-forced-exchange"
[ "${FORCED:-0}" = 1 ] && FX=""
for rep in $(seq 1 ${REPS:-2}); do
  for envset in ${ENVS:--}; do
    LOG=gpurun_out/ab/env_$(echo "$envset${BENCH_ARGS}" | tr -c 'a-zA-Z0-9_' '_').log
    ( [ "$envset" != "-" ] && export $(echo "$envset" | tr ',' ' ');
      timeout -k 10 200 python bench.py --steps ${STEPS:-50} --no-cpu-baseline $FX --wire-busbw ${BENCH_ARGS} > $LOG 2>&1 ) || { tail -5 $LOG; exit 1; }
    tail -1 $LOG | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms']; fx=d.get('forced_exchange') or {}; print('${BENCH_ARGS}', '$envset', d['config']['hook_path'], d['value'], 'fx', fx.get('value'), round(d['roofline']['avg_launch_us'],1) if d.get('roofline') else None, round(d['roofline']['hook']['device_us'],1) if d.get('roofline') else None)" | tee -a gpurun_out/ab/env_summary.txt
  done
done
