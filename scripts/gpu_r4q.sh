#!/bin/bash
# Round 4: pack chunks sized to the bucket (small buckets: more, smaller chunks): parity, A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4q gpurun_out/ab
rm -f gpurun_out/ab/summary.txt
ARCTOPK_LIB=allreducetopk_amd/lib/var/libarctopk_pk2048.so timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_arctopk.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4q/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r4q/tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/r4q/tests.log | head; exit $rc; }
for w in resnet18_ddp resnet50_mixed resnet18_conv headline; do
  BENCH_ARGS="--workload $w --steps 30" VARIANTS="pk1024 pk2048" bash scripts/gpu_ab_lib.sh || exit 1
done
