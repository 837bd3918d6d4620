#!/bin/bash
# bench.py on every workload (EF14), the headline bucket in all EF modes, the TopK / RandK
# baselines and the host-staged (NIC model) exchange.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/wl
: > gpurun_out/wl/all.jsonl
i=0
while read -r args; do
  [ -z "$args" ] && continue
  i=$((i+1))
  timeout -k 10 240 python bench.py $args --steps 20 --warmup 3 --no-cpu-baseline --no-forced-exchange \
      > gpurun_out/wl/w$i.log 2>&1 || { echo "bench [$args] failed"; tail -20 gpurun_out/wl/w$i.log; exit 1; }
  tail -1 gpurun_out/wl/w$i.log >> gpurun_out/wl/all.jsonl
  echo "[$args] done"
done <<LIST
--workload headline --ef ef14
--workload headline --ef ef21
--workload headline --ef noef
--workload headline --ef ef14 --host-staged
--workload llama_embed --ef ef14
--workload roberta_embed --ef ef14
--workload resnet18_conv --ef ef14
--workload resnet50_mixed --ef ef14
--workload llama_layer_mixed --ef ef14
--workload resnet18_ddp --ef ef14
--workload headline --ef ef14 --hook topk
--workload headline --ef ef14 --hook randk
--workload headline --ef ef14 --dtype bf16
--workload headline --ef ef14 --force-exchange
--workload resnet18_ddp --ef ef14 --force-exchange
--workload llama_embed --ef ef21 --force-exchange
${EXTRA_WL}
LIST
python scripts/wl_table.py gpurun_out/wl/all.jsonl
