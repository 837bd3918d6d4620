#!/bin/bash
# Round 4: window vs no window after the edge-bin register counts (A/B + per-kernel traces),
# and a kernel trace of the headline beside the emulated 8-rank wire.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4t gpurun_out/ab gpurun_out/r4e
rm -f gpurun_out/ab/summary.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_arctopk.py -m gpu -q -k "window_across_calls or end_to_end or degenerate or crowded" --timeout 120 --timeout-method thread > gpurun_out/r4t/sel2.log 2>&1
rc=$?; tail -2 gpurun_out/r4t/sel2.log; [ $rc -eq 0 ] || exit $rc
for w in resnet50_mixed resnet18_conv resnet18_ddp; do
  BENCH_ARGS="--workload $w --steps 30" VARIANTS="nowin" bash scripts/gpu_ab_lib.sh || exit 1
done
mkdir -p gpurun_out/r4e
for lib in product nowin; do
  if [ "$lib" = product ]; then L=""; else L="allreducetopk_amd/lib/var/libarctopk_$lib.so"; fi
  ARCTOPK_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r4e/tr_r50_$lib -o run -- \
    python3 bench.py --workload resnet50_mixed --steps 10 --warmup 3 --no-cpu-baseline --no-forced-exchange --wire-busbw --no-phase-events > gpurun_out/r4e/tr_r50_$lib.log 2>&1 || { tail -5 gpurun_out/r4e/tr_r50_$lib.log; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r4e/tr_wire -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-forced-exchange --wire-busbw 350 --no-phase-events > gpurun_out/r4e/tr_wire.log 2>&1 || { tail -5 gpurun_out/r4e/tr_wire.log; exit 1; }
tail -1 gpurun_out/r4e/tr_wire.log | cut -c1-300
