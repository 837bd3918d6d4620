#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
timeout -k 10 120 python3 scripts/sel_window_dbg.py 2>&1 | tee gpurun_out/r4d/selwin.log
