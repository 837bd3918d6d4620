#!/bin/bash
# Round-3 evidence at HEAD: GPU suite, default bench line, rocprofv3 headline (trace + PMC), all workloads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_r3prof.sh || exit 1
bash scripts/gpu_workloads.sh
