#!/bin/bash
# Rehearse the N>1 bench path on a 1-GPU box: 2 ranks share cuda:0 over gloo.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --backend gloo > gpurun_out/bench_rehearse2.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/bench_rehearse2.log; exit 1; }
grep '"metric"' gpurun_out/bench_rehearse2.log
