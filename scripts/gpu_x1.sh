#!/bin/bash
# Exchange path at N = 1: multirank / forced-exchange tests, smoke, step vs exchange bench, trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/x1
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py ${PYTEST_ARGS} -x -v --timeout 120 --timeout-method thread > gpurun_out/x1/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/x1/pytest.log | tail -20
if [ $rc -ne 0 ]; then grep -E "Error|assert|Traceback" -A3 gpurun_out/x1/pytest.log | head -60; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for mode in "" "--force-exchange"; do
  timeout -k 10 200 python bench.py --steps 50 --no-cpu-baseline $mode > gpurun_out/x1/bench$mode.log 2>&1 || { tail -20 gpurun_out/x1/bench$mode.log; exit 1; }
  tail -1 gpurun_out/x1/bench$mode.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['hook_path'], d['value'], d['ms_per_bucket'], d['phase_ms'], d['roofline']['frac'], d['roofline']['event_samples'], d['roofline']['hook'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/x1/trace -o run -- python3 bench.py --steps 20 --no-cpu-baseline --force-exchange > gpurun_out/x1/trace.log 2>&1 || { tail -20 gpurun_out/x1/trace.log; exit 1; }
tail -1 gpurun_out/x1/trace.log | cut -c1-200
find gpurun_out/x1/trace -name "*.csv" | head
