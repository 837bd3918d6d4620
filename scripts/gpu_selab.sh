#!/bin/bash
# Select-phase A/B: bench phase times of the select-heavy workloads under env settings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/selab
: > gpurun_out/selab/all.txt
for cfg in ${CONFIGS:-"X=0"}; do
  for w in ${WORKLOADS:-resnet50_mixed resnet18_conv llama_embed roberta_embed resnet18_ddp}; do
    env $cfg timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline \
        > gpurun_out/selab/$w.log 2>&1 || { echo "bench $w failed"; tail -5 gpurun_out/selab/$w.log; exit 1; }
    tail -1 gpurun_out/selab/$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d.get('phase_ms',{}); print('$cfg', '$w', d['value'], 'select', p.get('select'), 'dev', p.get('hook_device_total'))" | tee -a gpurun_out/selab/all.txt
  done
done
