#!/bin/bash
# Round-2 first GPU session: issue-cost microbenchmark, bench at HEAD, in-kernel
# clock stamps, rocprofv3 trace + PMC passes of the bench, and the per-workload
# kernel sweep.  Every GPU step has its own time limit; the first failure ends
# the script.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02a}
mkdir -p $O
timeout -k 10 120 scripts/microbench/issue2 > $O/issue2.txt 2>&1
echo "microbench done"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "bench done"
timeout -k 10 120 python scripts/clock_stamp.py --seconds 3 > $O/clock_linear_lqr.json 2> $O/clock.err
timeout -k 10 120 python scripts/clock_stamp.py --seconds 3 --motion sinusoidal --ctl lqi > $O/clock_sin_lqi.json 2>> $O/clock.err
echo "clock done"
timeout -k 10 300 python scripts/perf_sweep.py --n 65536 --motions linear,sinusoidal,circular,figure8,stationary,mixed \
  --ctl lqr,lqi --reps 3 > $O/sweep.jsonl 2> $O/sweep.err
echo "sweep done"
TAG=${TAG:-r02a} timeout -k 10 900 scripts/profile_session.sh > $O/profile.log 2>&1
echo "profile done"
