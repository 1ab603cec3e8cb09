#!/bin/bash
# Same-box alternating A/B of run_workload.py between library builds (GPU box):
#   CONFIGS="4 3" ROUNDS=2 [WL_ARGS="--episodes 65536"] scripts/ab_workloads.sh <lib.so|dir|tree> [...]
# One JSON line per (round, config, build) in gpurun_out/$TAG/ab_workloads.jsonl,
# each tagged with the build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-run}
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for c in ${CONFIGS:-4}; do
    for lib in "$@"; do
      L=$lib
      [ "$L" = tree ] && L=lqr-quadcopter-test_amd/quadtrack/_lib/libquadtrack.so
      [ -d "$L" ] && L=$L/libquadtrack.so
      L=$(realpath "$L")
      out=$(QUADTRACK_LIB=$L timeout -k 10 300 python -u scripts/run_workload.py --config $c --repeat ${REPEAT:-10} ${WL_ARGS:-} \
            2>> $O/ab_workloads.err) || exit 1
      echo "{\"build\": \"$lib\", \"round\": $r, \"line\": $out}" >> $O/ab_workloads.jsonl
    done
  done
done
