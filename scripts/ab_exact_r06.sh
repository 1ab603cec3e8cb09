#!/bin/bash
# Same-box A/B of the exact step's register pinning (round 6, DESIGN §3 "Exact
# step"): libraries built by scripts/ab_build.sh (build/ab/<name>) beside the
# in-tree build, alternated, scripts/flavour_timing.py's exact cases; the GPU
# tests on the in-tree build first.  VARIANTS, REPS; outputs gpurun_out/$TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab_exact}
mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
    || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for r in $(seq 1 ${REPS:-2}); do for v in ${VARIANTS:-pin0 tree}; do
  if [ $v = tree ]; then L=$PWD/lqr-quadcopter-test_amd/quadtrack/_lib/libquadtrack.so; else L=$PWD/build/ab/$v/libquadtrack.so; fi
  QUADTRACK_LIB=$L timeout -k 10 200 python scripts/flavour_timing.py --cases ${CASES:-exact exact_euler exact_rewards fast_yaw yaw0} \
    | sed "s/^/{\"lib\": \"$v\", \"rep\": $r, \"r\": /; s/$/}/" >> $O/ab_exact.jsonl || exit 1
done; done
