#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sbk
for v in keys2 keys1 stop1; do for w in resnet50 llama; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/sbk/$v$w -o run -- ./scripts/sb_$v $w 30 > /dev/null 2>&1 || exit 1
  echo "$v $w $(python3 scripts/kstats.py $(find gpurun_out/sbk/$v$w -name '*kernel_stats.csv' | head -1) 8 | grep k_arc_keys)"
done; done
