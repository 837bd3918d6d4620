#!/bin/bash
# A/B of library build variants through bench.py (ARCTOPK_LIB selects the library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
L=allreducetopk_amd/lib
for rep in 1 2; do
  for v in ${VARIANTS:-libarctopk.so}; do
    for ef in ${EFS:-ef14}; do
      ARCTOPK_LIB=$L/$v timeout -k 10 200 python bench.py --ef $ef --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab/$v.$ef.$rep.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/ab/$v.$ef.$rep.log; exit 1; }
      python - "$v $ef" gpurun_out/ab/$v.$ef.$rep.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["phase_ms"]
print(f"{sys.argv[1]:28s} value {d['value']:8.1f} GB/s  ms/bucket {d['ms_per_bucket']:.4f}  " +
      "  ".join(f"{k} {v*1e3:6.1f}" for k, v in ph.items()))
PY
    done
  done
done
