#!/bin/bash
# rocprofv3 kernel traces of bench.py for the workloads named in $WL (default: the weak ones).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
WL=${WL:-"llama_layer_mixed resnet18_conv resnet50_mixed"}
for w in $WL; do
  rm -rf gpurun_out/wlprof/$w
  mkdir -p gpurun_out/wlprof/$w
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/wlprof/$w -o run -- \
      python3 bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/wlprof/$w/log 2>&1 \
      || { echo "profile $w failed"; tail -20 gpurun_out/wlprof/$w/log; exit 1; }
  echo "$w done"
done
