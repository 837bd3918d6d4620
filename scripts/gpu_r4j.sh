#!/bin/bash
# Round 4: the ride's wait for an earlier packed all-reduce without the host event query (A/B),
# forced exchange, with the native host-time breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4j
for w in resnet18_ddp headline; do
  for rep in 1 2; do
    for lib in product noquery; do
      if [ "$lib" = product ]; then L=""; else L="allreducetopk_amd/lib/var/libarctopk_$lib.so"; fi
      ARCTOPK_LIB=$L ARCTOPK_HOST_TIMING=1 timeout -k 10 200 python3 bench.py --workload $w --force-exchange --steps 40 --no-cpu-baseline --no-phase-events --no-forced-exchange --wire-busbw > gpurun_out/r4j/$lib.log 2>&1 || { tail -5 gpurun_out/r4j/$lib.log; exit 1; }
      echo "== $w $lib $(tail -1 gpurun_out/r4j/$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])")"; grep native_step_host_us gpurun_out/r4j/$lib.log
    done
  done
done
