#!/bin/bash
# A/B of library variants beside the emulated 8-rank wire (350 GB/s busBW; BLOCKS workgroups per
# emulated collective): the step, the forced exchange and the wire line of each, interleaved.
# Lines go to stdout and gpurun_out/ab/wire_summary.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do
  for blocks in ${BLOCKS:-64 128}; do
    for lib in ${AB_LIBS:-product} ${VARIANTS}; do
      if [ "$lib" = product ]; then L=""; else L="allreducetopk_amd/lib/var/libarctopk_$lib.so"; fi
      LOG=gpurun_out/ab/wire_${lib}_${blocks}.log
      ARCTOPK_LIB=$L timeout -k 10 240 python bench.py --steps ${STEPS:-20} --no-cpu-baseline --no-phase-events \
          --wire-busbw ${BUSBW:-350} --wire-blocks $blocks ${BENCH_ARGS} > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
      tail -1 $LOG | python -c "import json,sys; d=json.loads(sys.stdin.read()); fx=d.get('forced_exchange') or {}; w=(d.get('emulated_wire') or [{}])[0]; print('${BENCH_ARGS}', '$lib', 'wg', $blocks, 'step', d['value'], 'fx', fx.get('value'), 'wire', w.get('per_gpu_value'), 'frac', w.get('frac_of_wire_ceiling'), 'ms/bucket', w.get('ms_per_bucket'))" | tee -a gpurun_out/ab/wire_summary.txt
    done
  done
done
