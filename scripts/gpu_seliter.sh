#!/bin/bash
# select iteration: parity subset, then rocprof traces of the select-heavy workloads
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "${PYTEST_K:-arctopk or configs or sparse}" > gpurun_out/pytest_sel.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/pytest_sel.log | head -30; tail -5 gpurun_out/pytest_sel.log; exit 1; }
tail -1 gpurun_out/pytest_sel.log
for wl in ${WLS:-resnet50_mixed resnet18_ddp}; do
  BENCH_ARGS="--workload $wl" bash scripts/trace_wl.sh $wl 2>&1 | head -40 || exit 1
done
