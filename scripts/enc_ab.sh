#!/bin/bash
# Encode A/B on one box: library variants x tile targets, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
L=allreducetopk_amd/lib
for rep in 1 2; do
for lib in libarctopk.so libarctopk_w4.so libarctopk_w5.so; do
  for tb in 1024 2048; do
    ARCTOPK_LIB=$L/$lib ARCTOPK_ENC_TARGET_BLOCKS=$tb TAG="${lib#libarctopk}:$tb" CASES="headline,1x[,4x[,llama layer,[32000" \
      timeout -k 10 120 python scripts/enc_probe.py 2>&1 | grep -v amdgpu || exit 1
  done
done
done
