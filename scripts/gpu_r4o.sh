#!/bin/bash
# Round 4: kernel traces beside the emulated wire: ResNet-50 mix (64 workgroups) and the headline
# with 128 workgroups.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4o
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r4o/tr_r50 -o run -- \
  python3 bench.py --workload resnet50_mixed --steps 10 --warmup 3 --no-cpu-baseline --no-forced-exchange --wire-busbw 350 --no-phase-events > gpurun_out/r4o/tr_r50.log 2>&1 || { tail -5 gpurun_out/r4o/tr_r50.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r4o/tr_h128 -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-forced-exchange --wire-busbw 350 --wire-blocks 128 --no-phase-events > gpurun_out/r4o/tr_h128.log 2>&1 || { tail -5 gpurun_out/r4o/tr_h128.log; exit 1; }
python3 scripts/wire_trace_summary.py gpurun_out/r4o/tr_r50 > gpurun_out/r4o/trace_wire_resnet50_mixed.txt
python3 scripts/wire_trace_summary.py gpurun_out/r4o/tr_h128 283 > gpurun_out/r4o/trace_wire_headline_128wg.txt
grep -h "all-reduce" gpurun_out/r4o/*.txt
