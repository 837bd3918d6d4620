#!/bin/bash
# Round-4 evidence at HEAD.  PART=a: the full GPU suite, the default bench line, rocprofv3 on the
# default bench command (trace + stats, FETCH_SIZE / WRITE_SIZE passes).  PART=b: every workload
# (EF14), the emulated 8-rank wire at 250 / 350 / 450 GB/s on the headline and the ResNet-50 mix,
# forced-exchange lines, the wire trace.  PART=c: SQ counter passes of the short-row workloads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4final
if [ "${PART:-a}" = a ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4final/pytest_gpu.log 2>&1
  rc=$?
  tail -3 gpurun_out/r4final/pytest_gpu.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc -- stopping"; grep -E "Error|FAIL|assert" gpurun_out/r4final/pytest_gpu.log | head -40; exit $rc; fi
  timeout -k 10 300 python bench.py > gpurun_out/r4final/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r4final/bench_default.log; exit 1; }
  tail -1 gpurun_out/r4final/bench_default.log
  bash scripts/profile.sh r4_headline_ef14 || exit 1
elif [ "${PART}" = b ]; then
  : > gpurun_out/r4final/wl.jsonl
  i=0
  while read -r args; do
    [ -z "$args" ] && continue
    i=$((i+1))
    timeout -k 10 240 python bench.py $args --steps 20 --warmup 3 --no-cpu-baseline \
        > gpurun_out/r4final/w$i.log 2>&1 || { echo "bench [$args] failed"; tail -20 gpurun_out/r4final/w$i.log; exit 1; }
    tail -1 gpurun_out/r4final/w$i.log >> gpurun_out/r4final/wl.jsonl
    echo "[$args] done"
  done <<LIST
--workload headline --ef ef14 --wire-busbw 250 350 450
--workload headline --ef ef21 --no-forced-exchange --wire-busbw
--workload headline --ef noef --no-forced-exchange --wire-busbw
--workload headline --ef ef14 --host-staged --wire-busbw
--workload llama_embed --ef ef14 --no-forced-exchange --wire-busbw
--workload roberta_embed --ef ef14 --no-forced-exchange --wire-busbw
--workload resnet18_conv --ef ef14 --no-forced-exchange --wire-busbw
--workload resnet50_mixed --ef ef14 --wire-busbw 250 350 450
--workload llama_layer_mixed --ef ef14 --no-forced-exchange --wire-busbw
--workload resnet18_ddp --ef ef14 --wire-busbw
--workload headline --ef ef14 --hook topk --no-forced-exchange --wire-busbw
--workload headline --ef ef14 --hook randk --no-forced-exchange --wire-busbw
--workload headline --ef ef14 --dtype bf16 --no-forced-exchange --wire-busbw
--workload llama_embed --ef ef21 --wire-busbw
LIST
  python scripts/wl_table.py gpurun_out/r4final/wl.jsonl > gpurun_out/r4final/workloads_table.txt
  cat gpurun_out/r4final/workloads_table.txt
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r4final/tr_wire -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-forced-exchange --wire-busbw 350 --no-phase-events > gpurun_out/r4final/tr_wire.log 2>&1 || { tail -5 gpurun_out/r4final/tr_wire.log; exit 1; }
  python3 scripts/wire_trace_summary.py gpurun_out/r4final/tr_wire 283 > gpurun_out/r4final/trace_wire_headline.txt
else
  WL="resnet18_conv resnet50_mixed headline:--dtype,bf16 headline:--ef,noef" bash scripts/gpu_r4counters.sh gpurun_out/r4final/pmc || exit 1
  for w in resnet18_conv resnet50_mixed headline_dtype_bf16 headline_ef_noef; do
    python3 scripts/sq_summary.py gpurun_out/r4final/pmc/$w > gpurun_out/r4final/sq_$w.txt
  done
fi
