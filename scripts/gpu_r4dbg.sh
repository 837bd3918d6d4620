#!/bin/bash
# Round 4 debug: the window select tests with the product library and with the window off;
# the short-row workloads' bench lines with the window off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
T="tests/test_gpu_arctopk.py -m gpu -k window_across_calls or end_to_end"
timeout -k 10 300 python -u -m pytest tests/test_gpu_arctopk.py -m gpu -v -k "window_across_calls or end_to_end" --timeout 120 --timeout-method thread > gpurun_out/r4d/product.log 2>&1
echo "product rc=$?"; grep -E "PASSED|FAILED|distinct rows" gpurun_out/r4d/product.log | head -20
ARCTOPK_LIB=allreducetopk_amd/lib/var/libarctopk_nowin.so timeout -k 10 300 python -u -m pytest tests/test_gpu_arctopk.py -m gpu -v -k "window_across_calls or end_to_end" --timeout 120 --timeout-method thread > gpurun_out/r4d/nowin.log 2>&1
echo "nowin rc=$?"; grep -E "PASSED|FAILED|distinct rows" gpurun_out/r4d/nowin.log | head -20
for w in resnet18_conv resnet50_mixed resnet18_ddp headline; do
  ARCTOPK_LIB=allreducetopk_amd/lib/var/libarctopk_nowin.so timeout -k 10 200 python3 bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4d/bench_$w.log 2>&1 || { tail -20 gpurun_out/r4d/bench_$w.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4d/bench_$w.log').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print('$w', d['value'], d['forced_exchange'] and d['forced_exchange']['value'], d['emulated_wire'], d['phase_ms'], (r.get('hook') or {}).get('frac'))"
done
