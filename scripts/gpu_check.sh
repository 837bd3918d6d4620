#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, a short bench. Each GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m3 -E "Marketing Name|gfx9" > gpurun_out/device.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 240 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc (crash/timeout) -- stopping"; exit $rc; fi
timeout -k 10 400 python bench.py --steps 30 --warmup 5 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -3 gpurun_out/bench.log
if [ -n "${HOST_PROFILE}" ]; then
  timeout -k 10 300 python scripts/host_profile.py > gpurun_out/host_profile.log 2>&1 || { echo "host profile failed"; tail -20 gpurun_out/host_profile.log; exit 1; }
  head -60 gpurun_out/host_profile.log
fi
