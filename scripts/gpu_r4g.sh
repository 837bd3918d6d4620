#!/bin/bash
# Round 4: parity of the vectorized mode-3 decode variant, A/B of decode / refine variants,
# SQ counter passes of the short-row workloads on the product library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g gpurun_out/ab
rm -f gpurun_out/ab/summary.txt
ARCTOPK_LIB=allreducetopk_amd/lib/var/libarctopk_vec3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_arctopk.py -m gpu -q -k "conv3x3 or resnet18 or resnet50 or end_to_end or golden or bf16" --timeout 120 --timeout-method thread > gpurun_out/r4g/vec3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4g/vec3_tests.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--workload resnet18_conv --steps 30" VARIANTS="vec3" bash scripts/gpu_ab_lib.sh || exit 1
BENCH_ARGS="--workload resnet50_mixed --steps 30" VARIANTS="refut16 refpre128" bash scripts/gpu_ab_lib.sh || exit 1
BENCH_ARGS="--workload resnet18_ddp --steps 30" VARIANTS="vec3 refut16" bash scripts/gpu_ab_lib.sh || exit 1
BENCH_ARGS="--workload headline --steps 30" VARIANTS="cap512 cap768 cap1024" bash scripts/gpu_ab_lib.sh || exit 1
# the encode grid cap beside the emulated 8-rank wire (is the collective queued behind the encode's blocks?)
for lib in product cap512 cap768; do
  if [ "$lib" = product ]; then L=""; else L="allreducetopk_amd/lib/var/libarctopk_$lib.so"; fi
  ARCTOPK_LIB=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-phase-events --no-forced-exchange --wire-busbw 350 > gpurun_out/r4g/wire_$lib.log 2>&1 || { tail -5 gpurun_out/r4g/wire_$lib.log; exit 1; }
  tail -1 gpurun_out/r4g/wire_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], [(x['per_gpu_value'], x['ms_per_bucket']) for x in d['emulated_wire']])"
done
# the pack's stop event: default (system-scope release) vs device-scope release, forced exchange
for w in resnet18_ddp headline; do
  for rep in 1 2; do
    for lib in product pkev pkev2; do
      if [ "$lib" = product ]; then L=""; else L="allreducetopk_amd/lib/var/libarctopk_$lib.so"; fi
      ARCTOPK_LIB=$L timeout -k 10 200 python3 bench.py --workload $w --force-exchange --steps 40 --no-cpu-baseline --no-phase-events --wire-busbw > gpurun_out/r4g/fx_${lib}_$w.log 2>&1 || { tail -5 gpurun_out/r4g/fx_${lib}_$w.log; exit 1; }
      tail -1 gpurun_out/r4g/fx_${lib}_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('forced $w $lib', d['value'], d['config'].get('hook_path'))"
    done
  done
done
bash scripts/gpu_r4counters.sh gpurun_out/r4g/pmc || exit 1
echo done
