#!/bin/bash
# Round 4: the N > 1 bench path rehearsed on one GPU (2 and 4 ranks share cuda:0 over gloo).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4reh
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2961$n bench.py --gpus $n --steps 10 --warmup 3 --backend gloo > gpurun_out/r4reh/bench_$n.log 2>&1 || { echo "rehearsal $n failed"; tail -30 gpurun_out/r4reh/bench_$n.log; exit 1; }
  grep '"metric"' gpurun_out/r4reh/bench_$n.log | cut -c1-400
done
