#!/bin/bash
# Build code-layout variants of libquadtrack (same results, -DQT_VARIANT=<v>)
# into build/var/<v>/ and time the rollout kernel of each with perf_sweep.py.
# Usage: scripts/variants.sh build "0 1 2 3"   (here, cross-compile)
#        scripts/variants.sh run   "0 1 2 3"   (GPU box)
cd "$(dirname "$0")/.."
mode=$1; shift
for v in ${1:-0 1}; do
  d=build/var/$v
  if [ "$mode" = build ]; then
    mkdir -p $d
    make -s -C lqr-quadcopter-test_amd OBJ=$(pwd)/$d/obj OUT=$(pwd)/$d DEFS="-DQT_VARIANT=$v ${EXTRA_FLAGS:-}" >/dev/null || exit 1
  else
    echo "variant=$v $(QUADTRACK_LIB=$(pwd)/$d/libquadtrack.so timeout -k 10 120 python scripts/perf_sweep.py --n 65536 --motions ${MOTIONS:-linear} --ctl ${CTLS:-lqr} --reps 5)" || exit 1
  fi
done
