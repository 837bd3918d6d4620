#!/bin/bash
# rocprofv3 kernel stats of the select harness per shape set
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sbprof
for w in ${SB_SETS:-resnet50 resnet18b0 llama headline}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/sbprof/$w -o run -- ./scripts/sb_full $w 30 > gpurun_out/sbprof/$w.log 2>&1 || { tail -5 gpurun_out/sbprof/$w.log; exit 1; }
  echo "== $w: $(grep select gpurun_out/sbprof/$w.log)"
  python3 scripts/kstats.py $(find gpurun_out/sbprof/$w -name "*kernel_stats.csv" | head -1) 8
done
