#!/bin/bash
# One GPU session: GPU tests, bench, clock stamps, kernel sweep (each step time-limited;
# the first failure ends the script).  TAG names the output dir; STEPS selects steps.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-run}
mkdir -p $O
for step in ${STEPS:-tests bench clock sweep}; do
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; } ;;
    bench) timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err ;;
    clock) timeout -k 10 120 python scripts/clock_stamp.py --seconds 2 > $O/clock_linear_lqr.json 2> $O/clock.err
           timeout -k 10 120 python scripts/clock_stamp.py --seconds 2 --motion sinusoidal --ctl lqi > $O/clock_sin_lqi.json 2>> $O/clock.err ;;
    sweep) timeout -k 10 300 python scripts/perf_sweep.py --n 65536 --motions ${MOTIONS:-linear,sinusoidal,circular,figure8,stationary,mixed} \
             --ctl ${CTLS:-lqr,lqi} --reps 3 > $O/sweep.jsonl 2> $O/sweep.err ;;
    workloads) for cfg in 3 5; do timeout -k 10 300 python scripts/run_workload.py --config $cfg >> $O/workloads.jsonl 2>> $O/workloads.err; done
               timeout -k 10 300 python scripts/run_workload.py --config 5 --episodes 131072 >> $O/workloads.jsonl 2>> $O/workloads.err
               timeout -k 10 300 python scripts/run_workload.py --config 4 --episodes 65536 >> $O/workloads.jsonl 2>> $O/workloads.err ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    profile) TAG=${TAG:-run} timeout -k 10 900 scripts/profile_session.sh > $O/profile.log 2>&1 ;;
    profw) TAG=${TAG:-run} timeout -k 10 900 scripts/profile_workloads.sh > $O/profw.log 2>&1 || { tail -20 $O/profw.log; exit 1; } ;;
    dropin) timeout -k 10 300 python scripts/dropin_loop.py > $O/dropin.jsonl 2> $O/dropin.err ;;
    dare) timeout -k 10 120 python scripts/dare_bench.py > $O/dare.jsonl 2> $O/dare.err ;;
  esac
  echo "$step done"
done
