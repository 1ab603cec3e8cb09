#!/bin/bash
# Same-box alternating A/B of the motion grouping on run_workload.py (GPU box):
# each variant is lib:order — a library (tree | a .so | a dir holding one) and
# core.GROUP_ORDER (QT_GROUP_ORDER).
#   VARIANTS="tree:0,1,2,3,4 tree:3,4,2,1,0" \
#   CONFIGS="5" ROUNDS=2 [WL_ARGS="--episodes 131072"] scripts/ab_grouping.sh
# One JSON line per (round, config, variant) in gpurun_out/$TAG/ab_grouping.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-run}
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for c in ${CONFIGS:-5}; do
    for v in ${VARIANTS:-tree:0,1,2,3,4 tree:3,4,2,1,0}; do
      IFS=: read -r lib order <<< "$v"
      L=$lib
      [ "$L" = tree ] && L=lqr-quadcopter-test_amd/quadtrack/_lib/libquadtrack.so
      [ -d "$L" ] && L=$L/libquadtrack.so
      L=$(realpath "$L")
      out=$(QUADTRACK_LIB=$L QT_GROUP_ORDER=$order timeout -k 10 300 \
            python -u scripts/run_workload.py --config $c --repeat ${REPEAT:-10} ${WL_ARGS:-} 2>> $O/ab_grouping.err) || exit 1
      echo "{\"variant\": \"$v\", \"round\": $r, \"args\": \"${WL_ARGS:-}\", \"line\": $out}" >> $O/ab_grouping.jsonl
    done
  done
done
