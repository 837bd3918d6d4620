#!/bin/bash
# Round evidence, part A: the full GPU suite, the default bench line (with the CPU baseline),
# and rocprofv3 on the default bench command (kernel trace + stats, then separate FETCH_SIZE /
# WRITE_SIZE passes).  Part B (PART=b): PMC passes on the short-row workloads and the
# forced-exchange headline trace.  Outputs under gpurun_out/; copied into profiles/<round>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${PART:-a}" = a ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc -- stopping"; grep -E "Error|FAIL|assert" gpurun_out/pytest_gpu.log | head -40; exit $rc; fi
  timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
  tail -1 gpurun_out/bench_default.log
  bash scripts/profile.sh headline_ef14 || exit 1
else
  BENCH_ARGS="--workload resnet18_conv --no-forced-exchange" bash scripts/profile.sh resnet18_conv_ef14 || exit 1
  BENCH_ARGS="--workload resnet50_mixed --no-forced-exchange" bash scripts/profile.sh resnet50_mixed_ef14 || exit 1
  BENCH_ARGS="--force-exchange" bash scripts/trace_wl.sh fx > gpurun_out/t_fx.txt 2>&1 || exit 1
  tail -25 gpurun_out/t_fx.txt
fi
