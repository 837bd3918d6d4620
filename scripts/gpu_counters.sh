#!/bin/bash
# Counter profile of bench workloads: per-kernel SQ instruction / wait counters (occupancy,
# issue vs latency) in rocprofv3 --pmc passes of their own (<= 8 SQ + 2 GRBM each); summarise
# with scripts/sq_summary.py OUT/<workload>.
# Usage: gpu_counters.sh [OUT] ; WL overrides the workloads (name or name:extra,args).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4c}
WL=${WL:-"resnet18_conv resnet50_mixed"}
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD"
LIST=$OUT/counters_list.txt
[ -s $LIST ] || timeout -k 10 60 rocprofv3 -L > $LIST 2>&1
keep() {  # the counters of $1 that this rocprofv3 lists
  local r=""
  for c in $1; do grep -qw "$c" $LIST && r="$r $c"; done
  echo $r
}
P1=$(keep "$P1"); P2=$(keep "$P2")
echo "pass 1: $P1"; echo "pass 2: $P2"
# WL entries: a workload name, or name:extra-args with commas for spaces (headline:--dtype,bf16)
for ent in $WL; do
  w=${ent%%:*}; extra=""; [ "$ent" != "$w" ] && extra=$(echo "${ent#*:}" | tr ',' ' ')
  tag=$(echo "$ent" | tr -c 'a-zA-Z0-9_\n' '_' | sed 's/__*/_/g; s/_$//')
  w_dir=$OUT/$tag
  mkdir -p $w_dir
  ARGS="--workload $w $extra --steps 6 --warmup 3 --no-cpu-baseline --no-forced-exchange --no-phase-events --wire-busbw"
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -T --output-format csv -d $w_dir/p$i -o run -- \
        python3 bench.py $ARGS > $w_dir/p$i.log 2>&1 || { echo "pmc pass $i of $ent failed"; tail -5 $w_dir/p$i.log; exit 1; }
    echo "$ent pass $i done"
  done
done
