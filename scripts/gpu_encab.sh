#!/bin/bash
# Encode rework: quick parity subset, then library-variant and tile-count A/B through bench.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "phases or headline or golden or configs" > gpurun_out/pytest_enc.log 2>&1 || { tail -30 gpurun_out/pytest_enc.log; exit 1; }
tail -1 gpurun_out/pytest_enc.log
VARIANTS="libarctopk.so libarctopk_old.so libarctopk_u4w5.so libarctopk_u8w3.so" bash scripts/gpu_ab.sh || exit 1
KNOBS="ARCTOPK_ENC_TARGET_BLOCKS=4096 ARCTOPK_ENC_TARGET_BLOCKS=1024" bash scripts/gpu_envab2.sh
