#!/bin/bash
# copy-stream HW queue A/B: v_waits and wall per call under the plain hook loop (no profiler)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for v in "X=0" "GPU_MAX_HW_QUEUES=8" "ARCTOPK_COPY_PRIORITY=-1"; do
  echo "== $v"; env $v ONLY_ON=1 timeout -k 10 120 python scripts/prestage_probe.py 2>&1 | grep "host enqueue" || exit 1
done
