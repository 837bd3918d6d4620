#!/bin/bash
# Round-3 measurement pass: every workload (step and exchange paths), then rocprofv3 trace +
# FETCH/WRITE PMC passes of the short-row workloads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
EXTRA_WL="--workload headline --ef ef14 --force-exchange
--workload headline --ef ef21 --force-exchange
--workload resnet18_ddp --ef ef14 --force-exchange
--workload llama_embed --ef ef21 --force-exchange
--workload resnet50_mixed --ef ef14 --force-exchange" bash scripts/gpu_workloads.sh || exit 1
for wl in resnet18_conv resnet50_mixed; do
  BENCH_ARGS="--workload $wl" bash scripts/profile.sh r03_$wl > /dev/null 2>&1 || { echo "profile $wl failed"; exit 1; }
  echo "== $wl"; grep -E "k_pack|k_decode|k_encode|k_arc|k_select" gpurun_out/prof_r03_$wl/summary.txt
done
