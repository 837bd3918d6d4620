#!/bin/bash
# Round 4: host-time breakdown of the exchange step (native parts) on ResNet-18 DDP and the
# headline, forced exchange vs step path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4i
for w in resnet18_ddp headline; do
  for fx in "" "--force-exchange"; do
    ARCTOPK_HOST_TIMING=1 timeout -k 10 200 python3 bench.py --workload $w $fx --steps 30 --no-cpu-baseline --no-phase-events --no-forced-exchange --wire-busbw > gpurun_out/r4i/ht_${w}${fx}.log 2>&1 || { tail -5 gpurun_out/r4i/ht_${w}${fx}.log; exit 1; }
    echo "== $w $fx"; grep -E "host_us_per_call|native_step_host_us" gpurun_out/r4i/ht_${w}${fx}.log
    tail -1 gpurun_out/r4i/ht_${w}${fx}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
  done
done
