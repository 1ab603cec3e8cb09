#!/bin/bash
# A/B timing of the rollout kernel between library builds (GPU box):
#   scripts/ab.sh <lib.so> [<lib.so> ...]   (the in-tree build if "tree")
# Each line: the perf_sweep JSON of that build (median of 5, 3,000 steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in "$@"; do
  [ "$lib" = tree ] && lib=lqr-quadcopter-test_amd/quadtrack/_lib/libquadtrack.so
  [ -d "$lib" ] && lib=$lib/libquadtrack.so
  lib=$(realpath "$lib")
  echo "== $lib"
  QUADTRACK_LIB=$lib timeout -k 10 300 python scripts/perf_sweep.py --n ${NS:-65536} --motions ${MOTIONS:-linear} \
    --ctl ${CTLS:-lqr} --reps 5 || exit 1
done
