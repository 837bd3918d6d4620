#!/bin/bash
# Perf pass: per-kernel microbench, host profile, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/kernel_bench.py > gpurun_out/kernel_bench.log 2>&1 || { echo "kernel_bench failed"; tail -30 gpurun_out/kernel_bench.log; exit 1; }
grep -v -E "^\[|Warning|amdgpu.ids" gpurun_out/kernel_bench.log
if [ -n "${RESNET}" ]; then
  SHAPES=resnet18 timeout -k 10 300 python scripts/kernel_bench.py > gpurun_out/kernel_bench_resnet.log 2>&1 || { echo "kernel_bench resnet failed"; tail -30 gpurun_out/kernel_bench_resnet.log; exit 1; }
  grep -v -E "^\[|Warning|amdgpu.ids" gpurun_out/kernel_bench_resnet.log
fi
timeout -k 10 300 python scripts/host_profile.py > gpurun_out/host_profile.log 2>&1 || { echo "host profile failed"; tail -20 gpurun_out/host_profile.log; exit 1; }
grep -E "us/step|hits|manual_seed|all_reduce" gpurun_out/host_profile.log
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --cpu-seconds 3 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
