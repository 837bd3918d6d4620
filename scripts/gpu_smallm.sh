#!/bin/bash
# small-m paths: parity subset, then the small-m workloads through bench.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/wl
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "arctopk or configs" > gpurun_out/pytest_sm.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/pytest_sm.log | head -30; tail -5 gpurun_out/pytest_sm.log; exit 1; }
tail -1 gpurun_out/pytest_sm.log
for wl in resnet50_mixed resnet18_ddp resnet18_conv headline; do
  timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/wl/sm_$wl.log 2>&1 || { tail -20 gpurun_out/wl/sm_$wl.log; exit 1; }
  python - gpurun_out/wl/sm_$wl.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ph = d["phase_ms"]
print(f"{d['config']['workload'][:60]:60s} {d['value']:8.1f} GB/s  " + "  ".join(f"{k} {v*1e3:6.1f}" for k, v in ph.items()), flush=True)
PY
done
