#!/bin/bash
# Select-focused GPU pass: parity tests, select diagnostics, a per-kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf gpurun_out/selp
mkdir -p gpurun_out/selp
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 240 -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc -- stopping"; exit $rc; fi
timeout -k 10 120 python scripts/sel_diag.py > gpurun_out/sel_diag.log 2>&1 || { echo "diag failed"; tail -20 gpurun_out/sel_diag.log; exit 1; }
cat gpurun_out/sel_diag.log | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/selp -o run -- python3 scripts/sel_profile.py > gpurun_out/selp/log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/selp/log; exit 1; }
echo "profile ok"
