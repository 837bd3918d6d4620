#!/bin/bash
# Round evidence, part B: short-row PMC passes, the forced-exchange trace, then every workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PART=b bash scripts/gpu_r3prof.sh || exit 1
bash scripts/gpu_workloads.sh
