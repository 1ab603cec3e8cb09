#!/bin/bash
# Same-box alternating A/B of core.motion_groups' mixed tail (QT_MIXED_TAIL=0/1)
# on run_workload.py (GPU box):
#   CONFIGS="5" ROUNDS=2 [WL_ARGS="--episodes 131072"] scripts/ab_mixed_tail.sh
# One JSON line per (round, config, setting) in gpurun_out/$TAG/ab_mixed_tail.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-run}
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for c in ${CONFIGS:-5}; do
    for t in 0 1; do
      out=$(QT_MIXED_TAIL=$t timeout -k 10 300 python -u scripts/run_workload.py --config $c --repeat ${REPEAT:-10} \
            ${WL_ARGS:-} 2>> $O/ab_mixed_tail.err) || exit 1
      echo "{\"mixed_tail\": $t, \"round\": $r, \"args\": \"${WL_ARGS:-}\", \"line\": $out}" >> $O/ab_mixed_tail.jsonl
    done
  done
done
