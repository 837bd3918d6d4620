#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/seq
mkdir -p $O
for m in ${MODES:-full enc}; do
  SEQ=$m timeout -k 10 120 rocprofv3 --kernel-trace -T --output-format csv -d $O/$m -o run -- python3 scripts/seq_probe.py > $O/$m.log 2>&1 || { tail -20 $O/$m.log; exit 1; }
  echo "== $m"; python3 scripts/gaps.py $(find $O/$m -name "*kernel_trace.csv" | head -1)
done
if [ -n "$HOOK" ]; then
  ONLY_ON=1 timeout -k 10 120 rocprofv3 --kernel-trace -T --output-format csv -d $O/hook -o run -- python3 scripts/prestage_probe.py > $O/hook.log 2>&1 || { tail -20 $O/hook.log; exit 1; }
  grep "host enqueue" $O/hook.log
  echo "== hook"; python3 scripts/gaps.py $(find $O/hook -name "*kernel_trace.csv" | head -1)
fi
