#!/bin/bash
# A/B/C of library builds under build/ab/: rollout timing (perf_sweep) on the
# bench workload and config 3's, then the clock-stamp builds' cycles per step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab3.jsonl
for v in ${VARS:-A B C}; do
  for mc in "linear lqr" "sinusoidal lqi"; do
    set -- $mc
    echo "{\"var\": \"$v\", \"motion\": \"$1\", \"ctl\": \"$2\"}" >> gpurun_out/ab3.jsonl
    QUADTRACK_LIB=$(pwd)/build/ab/$v/libquadtrack.so timeout -k 10 120 python scripts/perf_sweep.py --n 65536 \
      --motions $1 --ctl $2 --reps 7 >> gpurun_out/ab3.jsonl 2>> gpurun_out/ab3.err || exit 3
  done
done
for v in ${VARS:-A B C}; do
  for mc in "linear lqr" "sinusoidal lqi"; do
    set -- $mc
    echo "{\"stamp\": \"$v\", \"motion\": \"$1\"}" >> gpurun_out/ab3.jsonl
    QUADTRACK_LIB=$(pwd)/build/ab/${v}s/libquadtrack.so timeout -k 10 120 python scripts/clock_stamp.py --motion $1 \
      --ctl $2 --seconds 2 >> gpurun_out/ab3.jsonl 2>> gpurun_out/ab3.err || exit 4
  done
done
cut -c1-400 gpurun_out/ab3.jsonl
