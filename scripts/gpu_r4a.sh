#!/bin/bash
# Round-4 first call: the available counters, the default bench line at HEAD, the
# short-row workloads' bench lines and their SQ counter passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a/pmc
timeout -k 10 60 rocprofv3 -L > gpurun_out/r4a/pmc/counters_list.txt 2>&1 || echo "counter list failed"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4a/bench_default.log 2>&1 || { tail -20 gpurun_out/r4a/bench_default.log; exit 1; }
tail -1 gpurun_out/r4a/bench_default.log
for w in resnet18_conv resnet50_mixed resnet18_ddp; do
  timeout -k 10 200 python3 bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4a/bench_$w.log 2>&1 || { tail -20 gpurun_out/r4a/bench_$w.log; exit 1; }
  tail -1 gpurun_out/r4a/bench_$w.log | cut -c1-400
done
bash scripts/gpu_r4counters.sh gpurun_out/r4a/pmc
