#!/bin/bash
# Round 4: GPU tests (new first, then the suite), then the short-row workloads' bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash scripts/gpu_r4tests.sh || exit 1
mkdir -p gpurun_out/r4b
for w in resnet18_conv resnet50_mixed resnet18_ddp headline; do
  timeout -k 10 200 python3 bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4b/bench_$w.log 2>&1 || { tail -20 gpurun_out/r4b/bench_$w.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4b/bench_$w.log').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print('$w', d['value'], d['forced_exchange'] and d['forced_exchange']['value'], d['phase_ms'], (r.get('hook') or {}).get('frac'))"
done
