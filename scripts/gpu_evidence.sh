#!/bin/bash
# The round's profile evidence on one box, at the library being committed: for each entry of
# PROFILES ("tag:bench args with commas for spaces"), scripts/profile.sh (kernel trace + stats,
# FETCH_SIZE and WRITE_SIZE passes) and the files bench.py reads back, renamed under
# gpurun_out/evidence/: rocprof_summary_<tag>.txt and pmc_<tag>.json.  CALL_KERNELS is set per
# entry (one launch per hook call) for the per-call bytes.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/evidence
mkdir -p $OUT
for ent in ${PROFILES}; do
  tag=${ent%%:*}; args=""; [ "$ent" != "$tag" ] && args=$(echo "${ent#*:}" | tr ',' ' ')
  case "$args" in *--hook*) export CALL_KERNELS=k_scatter_first ;; *) export CALL_KERNELS=k_encode,k_encode_short,k_encode_carry ;; esac
  BENCH_ARGS="$args" bash scripts/profile.sh ev_$tag > $OUT/profile_$tag.log 2>&1 || { echo "profile $tag failed"; tail -20 $OUT/profile_$tag.log; exit 1; }
  cp gpurun_out/prof_ev_$tag/summary.txt $OUT/rocprof_summary_$tag.txt
  cp gpurun_out/prof_ev_$tag/pmc_per_launch.json $OUT/pmc_$tag.json
  grep -h '"metric"' gpurun_out/prof_ev_$tag/bench_trace.log > $OUT/bench_$tag.json
  echo "$tag done"
done
