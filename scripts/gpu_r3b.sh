#!/bin/bash
# parity tests touching the select/decode paths, then the workload sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
K="configs or multirank or end_to_end or golden or phases" bash scripts/gpu_k.sh > /dev/null || { grep -E "FAILED|Error|assert" gpurun_out/pytest_k.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_k.log
EXTRA_WL="--workload headline --ef ef14 --force-exchange
--workload resnet18_ddp --ef ef14 --force-exchange
--workload llama_embed --ef ef21 --force-exchange" bash scripts/gpu_workloads.sh
