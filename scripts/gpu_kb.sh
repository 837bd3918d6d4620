#!/bin/bash
# Per-kernel timings (kernel_bench.py) + select thread-count switch via bench.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/kernel_bench.py > gpurun_out/kb.log 2>&1 || { tail -20 gpurun_out/kb.log; exit 1; }
cat gpurun_out/kb.log
KNOBS="ARCTOPK_SEL_BIG_ROWS=1024 ARCTOPK_ENC_TARGET_BLOCKS=1536 ARCTOPK_ENC_TARGET_BLOCKS=3072" bash scripts/gpu_envab2.sh
