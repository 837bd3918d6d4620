#!/bin/bash
# projection source A/B (device vs host) on the headline and small-bucket workloads
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/proj
for rep in 1 2; do for wl in headline resnet18_ddp resnet50_mixed; do for mode in device host; do
  ARCTOPK_PROJECTIONS=$mode ARCTOPK_HOST_TIMING=1 timeout -k 10 200 python bench.py --workload $wl --steps 30 --warmup 5 --no-cpu-baseline --no-phase-events > gpurun_out/proj/$wl.$mode.$rep.log 2>&1 || { tail -20 gpurun_out/proj/$wl.$mode.$rep.log; exit 1; }
  python3 - gpurun_out/proj/$wl.$mode.$rep.log $mode <<'PY'
import json, sys
lines = open(sys.argv[1]).read().splitlines()
d = json.loads([l for l in lines if l.startswith("{")][-1])
h = json.loads([l for l in lines if l.startswith("host_us")][-1].split(" ", 1)[1])
print(f"{d['config']['workload'][:50]:50s} {sys.argv[2]:6s} {d['value']:8.1f} GB/s  {d['ms_per_bucket']*1e3:6.1f} us/bucket  host {sum(h.values()):5.1f} us/call", flush=True)
PY
done; done; done
