#!/bin/bash
# host cost per hook call: breakdown (ARCTOPK_HOST_TIMING) and the host_profile loops
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/host
for wl in resnet18_ddp headline; do
  ARCTOPK_HOST_TIMING=1 timeout -k 10 200 python bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline --no-phase-events > gpurun_out/host/bench_$wl.log 2>&1 || { tail -20 gpurun_out/host/bench_$wl.log; exit 1; }
  grep host_us gpurun_out/host/bench_$wl.log
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/host/bench_$wl.log') if l.startswith('{')][-1]); print('$wl', d['value'], d['ms_per_bucket'])"
  WORKLOAD=$wl timeout -k 10 200 python scripts/host_profile.py > gpurun_out/host/prof_$wl.log 2>&1 || { tail -20 gpurun_out/host/prof_$wl.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/host/prof_$wl.log | head -30
done
