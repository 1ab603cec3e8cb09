#!/bin/bash
# Build timing-only ablation variants of libquadtrack (wrong results by design)
# into build/abl/<bits>/ and time the rollout kernel of each with perf_sweep.py.
# Usage: scripts/ablate.sh build "0 1 2 4 8 16"   (here, cross-compile)
#        scripts/ablate.sh run   "0 1 2 4 8 16"   (GPU box)
cd "$(dirname "$0")/.."
mode=$1; shift
for b in ${1:-0 1 2 4 8 16 31}; do
  d=build/abl/$b
  if [ "$mode" = build ]; then
    mkdir -p $d
    make -s -C lqr-quadcopter-test_amd OBJ=$(pwd)/$d/obj OUT=$(pwd)/$d DEFS="-DQT_ABLATE=$b" >/dev/null || exit 1
  else
    echo "ablate=$b $(QUADTRACK_LIB=$(pwd)/$d/libquadtrack.so timeout -k 10 120 python scripts/perf_sweep.py --n 65536 --motions linear --ctl lqr --reps 3)"
  fi
done
