#!/bin/bash
# One GPU iteration: encode A/B probe (library variants), GPU parity tests, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -x scripts/stream_probe ] && [ -z "${SKIP_PROBE}" ]; then
  for il in 0 1; do
    ARCTOPK_ENC_INTERLEAVE=$il timeout -k 10 120 ./scripts/stream_probe > gpurun_out/probe_il$il.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/probe_il$il.log; exit 1; }
    echo "== interleave=$il"; grep -E "library|nt both" gpurun_out/probe_il$il.log | grep -v "chunk"
  done
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; grep -E "Error|error|FAIL|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
