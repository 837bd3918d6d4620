#!/bin/bash
# (historical: the CU partition and codec pipelining it measured were reverted, see
#  profiles/r04/experiments_not_kept.txt; the environment switches it sets no longer exist)
# Round 4: CU partition of the exchange path (GroupTopKState.exchange_cus) beside the emulated
# 8-rank wire: parity, wire lines at several reserved-CU counts, a kernel trace; host timing of
# the forced-exchange ResNet-18 DDP buckets.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4f
timeout -k 10 300 python -u -m pytest tests/test_gpu_exchange_failures.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4f/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4f/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_arctopk.py -m gpu -q -k "resnet50 or conv3x3 or window or crowded or degenerate" --timeout 120 --timeout-method thread > gpurun_out/r4f/tests_sel.log 2>&1
rc=$?; tail -2 gpurun_out/r4f/tests_sel.log; [ $rc -eq 0 ] || exit $rc
for w in headline resnet50_mixed resnet18_ddp; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-phase-events --wire-busbw 350 --wire-xcu 0 16 32 64 > gpurun_out/r4f/wire_$w.log 2>&1 || { tail -5 gpurun_out/r4f/wire_$w.log; exit 1; }
  python3 - "$w" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r4f/wire_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[1], "value", d["value"], "forced", (d.get("forced_exchange") or {}).get("value"))
for x in d.get("emulated_wire") or []:
    print("   xcu", x["exchange_cus"], "per_gpu", x["per_gpu_value"], "ms/bucket", x["ms_per_bucket"])
PY
done
ARCTOPK_XCU=32 timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r4f/tr_wire32 -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-forced-exchange --wire-busbw 350 --wire-xcu 32 --no-phase-events > gpurun_out/r4f/tr_wire32.log 2>&1 || { tail -5 gpurun_out/r4f/tr_wire32.log; exit 1; }
ARCTOPK_HOST_TIMING=1 timeout -k 10 240 python3 bench.py --workload resnet18_ddp --force-exchange --steps 30 --no-cpu-baseline --wire-busbw --no-phase-events > gpurun_out/r4f/ht_r18.log 2>&1 || { tail -5 gpurun_out/r4f/ht_r18.log; exit 1; }
ARCTOPK_HOST_TIMING=1 timeout -k 10 240 python3 bench.py --workload resnet18_ddp --steps 30 --no-cpu-baseline --no-forced-exchange --wire-busbw --no-phase-events > gpurun_out/r4f/ht_r18_step.log 2>&1 || { tail -5 gpurun_out/r4f/ht_r18_step.log; exit 1; }
echo done
