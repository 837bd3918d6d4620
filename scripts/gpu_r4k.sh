#!/bin/bash
# Round 4: parity of the paired last-step decode (exchange-path GPU tests), then forced-exchange
# lines with the native host-time breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4k
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_exchange_failures.py tests/test_gpu_configs.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r4k/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4k/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/r4k/tests.log | head -20; exit $rc; }
for w in resnet18_ddp headline resnet50_mixed; do
  ARCTOPK_HOST_TIMING=1 timeout -k 10 200 python3 bench.py --workload $w --steps 40 --no-cpu-baseline --no-phase-events --wire-busbw > gpurun_out/r4k/$w.log 2>&1 || { tail -5 gpurun_out/r4k/$w.log; exit 1; }
  echo "== $w"; grep native_step_host_us gpurun_out/r4k/$w.log
  tail -1 gpurun_out/r4k/$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('step', d['value'], 'forced', d['forced_exchange']['value'])"
done
