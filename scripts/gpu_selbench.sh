#!/bin/bash
# select-only timing of the harness variants (scripts/sb_*) on several shape sets
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${SB_VARIANTS:-full nosmall stop1 keys1 keys2 smallonly}; do
  for w in ${SB_SETS:-resnet50 resnet18b0 resnet18b1 llama roberta headline}; do
    printf "%-10s " $v
    timeout -k 5 60 ./scripts/sb_$v $w 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
