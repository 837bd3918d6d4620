#!/bin/bash
# Round 4: smoke() on cuda:0, then the default bench line again (PMC file of this library committed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4smoke/smoke.log 2>&1 || { tail -20 gpurun_out/r4smoke/smoke.log; exit 1; }
tail -1 gpurun_out/r4smoke/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r4smoke/bench_default.log 2>&1 || { tail -20 gpurun_out/r4smoke/bench_default.log; exit 1; }
tail -1 gpurun_out/r4smoke/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['frac'], r['traffic_lib_match'], d['forced_exchange']['value'], d['emulated_wire'][0]['per_gpu_value'])"
