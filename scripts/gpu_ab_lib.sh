#!/bin/bash
# A/B of library variants on one box: bench.py (args in BENCH_ARGS) with each lib, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for lib in product ${VARIANTS}; do
    if [ "$lib" = product ]; then L=""; else L="allreducetopk_amd/lib/var/libarctopk_$lib.so"; fi
    ARCTOPK_LIB=$L timeout -k 10 200 python bench.py --steps 50 --no-cpu-baseline --no-forced-exchange ${BENCH_ARGS} > gpurun_out/ab/$lib.log 2>&1 || { tail -5 gpurun_out/ab/$lib.log; exit 1; }
    tail -1 gpurun_out/ab/$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms']; print('$lib', d['config']['hook_path'], d['value'], round(d['roofline']['avg_launch_us'],1), round(d['roofline']['hook']['device_us'],1), {k: round(v*1e3,1) for k,v in p.items()})"
  done
done
