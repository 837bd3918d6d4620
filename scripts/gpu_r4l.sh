#!/bin/bash
# Round 4: the emulated wire with more workgroups (32 cannot reach the 350 GB/s pace even alone:
# ~12 GB/s of copy per workgroup); encode block target of the G-only / bf16 tile table (A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4l gpurun_out/ab
rm -f gpurun_out/ab/summary.txt
for b in 64 128; do
  for w in headline resnet50_mixed; do
    timeout -k 10 300 python3 bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-phase-events --no-forced-exchange --wire-busbw 250 350 450 --wire-blocks $b > gpurun_out/r4l/wire_${w}_$b.log 2>&1 || { tail -5 gpurun_out/r4l/wire_${w}_$b.log; exit 1; }
    tail -1 gpurun_out/r4l/wire_${w}_$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w blocks $b', d['value'], [(x['busbw_gbs'], x['per_gpu_value'], x['ms_per_bucket']) for x in d['emulated_wire']])"
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r4l/tr_wire64 -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-forced-exchange --wire-busbw 350 --wire-blocks 64 --no-phase-events > gpurun_out/r4l/tr_wire64.log 2>&1 || { tail -5 gpurun_out/r4l/tr_wire64.log; exit 1; }
python3 scripts/wire_trace_summary.py gpurun_out/r4l/tr_wire64 283 > gpurun_out/r4l/trace_wire64.txt
for args in "--ef noef" "--dtype bf16" "--ef ef14"; do
  BENCH_ARGS="--workload headline $args --steps 30" VARIANTS="t3072 t4096" bash scripts/gpu_ab_lib.sh || exit 1
done
