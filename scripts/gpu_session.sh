#!/bin/bash
# One GPU session (run under gpurun): the steps named in STEPS, in order, each
# under its own time limit; the first failure ends the session.  Outputs under
# gpurun_out/$TAG/.
#
#   STEPS="tests smoke bench" TAG=r03x bash scripts/gpu_session.sh
#
# steps:
#   tests      pytest -m gpu (PYTEST_ARGS narrows it)
#   smoke      __graft_entry__.smoke()
#   bench      bench.py with the driver's defaults (BENCH_ARGS adds flags)
#   benchab    bench.py at --steps 20 --warmup 5 and --steps 100 --warmup 20 (steadiness)
#   workloads  scripts/run_workload.py for CONFIGS (default "3 4 5")
#   dare       scripts/dare_bench.py (structured + dense DARE throughput)
#   ab         scripts/ab.sh on LIBS (library builds, "tree" = in-tree) via perf_sweep
#   clock      in-kernel clock stamps (scripts/clock_stamp.py; needs `make stamp`)
#   profile    rocprofv3 trace + PMC passes of the bench (scripts/profile_session.sh)
#   profw      the same for the config-3/5 workloads (scripts/profile_workloads.sh)
#   prof       rocprofv3 trace + PMC_SETS passes of PROF_CMD (scripts/prof.sh)
#   riders     config 5's 8-GPU shards timed on one GPU (run_workload.py --shard r/8, RANKS, default 0-7)
#              with stationary riders and without (QT_RIDERS=0), alternating ALT times; then the
#              whole config both ways
#   small      the fused rollout at small per-GPU batches (scripts/small_batch.py), with a kernel trace
#   pairing    config 5's 8-GPU shards with the resident set's rounds paired and without
#              (QT_PAIR_ROUNDS=0), alternating ALT times over RANKS
#   shards     the per-rank shards of configs 4 and 5 for W = 1, 2, 4, 8 ranks (first and last rank),
#              timed on one GPU (run_workload.py --shard): the predicted 1/2/4/8-GPU table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-run}
mkdir -p $O
fail() { echo "step $1 failed"; tail -40 "$2"; exit 1; }
for step in ${STEPS:-tests smoke bench}; do
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
             > $O/tests.log 2>&1 || fail tests $O/tests.log
           tail -3 $O/tests.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
           tail -1 $O/smoke.log ;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err ;;
    benchab) timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20_w5.json 2> $O/benchab.err || fail benchab $O/benchab.err
             timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_s100_w20.json 2>> $O/benchab.err \
               || fail benchab $O/benchab.err ;;
    workloads) for c in ${CONFIGS:-3 4 5}; do
                 timeout -k 10 300 python -u scripts/run_workload.py --config $c --repeat 10 >> $O/workloads.jsonl 2>> $O/workloads.err \
                   || fail workloads $O/workloads.err
               done ;;
    dare) timeout -k 10 300 python scripts/dare_bench.py ${DARE_ARGS:-} > $O/dare.jsonl 2> $O/dare.err || fail dare $O/dare.err ;;
    ab) timeout -k 10 600 bash scripts/ab.sh ${LIBS:-tree} > $O/ab.log 2>&1 || fail ab $O/ab.log ;;
    clock) timeout -k 10 120 python scripts/clock_stamp.py --seconds 2 > $O/clock_linear_lqr.json 2> $O/clock.err || fail clock $O/clock.err
           timeout -k 10 120 python scripts/clock_stamp.py --seconds 2 --motion sinusoidal --ctl lqi > $O/clock_sin_lqi.json \
             2>> $O/clock.err || fail clock $O/clock.err ;;
    profile) TAG=${TAG:-run} timeout -k 10 900 bash scripts/profile_session.sh > $O/profile.log 2>&1 || fail profile $O/profile.log ;;
    profw) TAG=${TAG:-run} timeout -k 10 900 bash scripts/profile_workloads.sh > $O/profw.log 2>&1 || fail profw $O/profw.log ;;
    prof) TAG=${TAG:-run} timeout -k 10 900 bash scripts/prof.sh ${PROF_CMD} > $O/prof.log 2>&1 || fail prof $O/prof.log ;;
    riders) for a in $(seq 1 ${ALT:-1}); do for r in ${RANKS:-0 1 2 3 4 5 6 7}; do for rd in 1 0; do
              QT_RIDERS=$rd timeout -k 10 120 python -u scripts/run_workload.py --config 5 --shard $r/8 --repeat 10 \
                >> $O/riders.jsonl 2>> $O/riders.err || fail riders $O/riders.err
            done; done; done
            for rd in 1 0; do
              QT_RIDERS=$rd timeout -k 10 200 python -u scripts/run_workload.py --config 5 --repeat 10 \
                >> $O/riders_full.jsonl 2>> $O/riders.err || fail riders $O/riders.err
            done ;;
    small) timeout -k 10 300 python -u scripts/small_batch.py > $O/small_batch.jsonl 2> $O/small.err || fail small $O/small.err
           timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/small_trace -o run -- \
             python3 scripts/small_batch.py --reps 10 > $O/small_trace.log 2>&1 || fail small $O/small_trace.log
           cp $(find $O/small_trace -name "*kernel_stats.csv" | head -1) $O/small_kernel_stats.csv
           cp $(find $O/small_trace -name "*kernel_trace.csv" | head -1) $O/small_kernel_trace.csv ;;
    pairing) for a in $(seq 1 ${ALT:-1}); do for r in ${RANKS:-0 1 2 3 4 5 6 7}; do for pr in 1 0; do
               QT_PAIR_ROUNDS=$pr timeout -k 10 120 python -u scripts/run_workload.py --config 5 --shard $r/8 --repeat 10 \
                 | sed "s/^/{\"pair_rounds\": $pr, \"r\": /; s/$/}/" >> $O/pairing.jsonl 2>> $O/pairing.err \
                 || fail pairing $O/pairing.err
             done; done; done ;;
    shards) for c in 4 5; do for w in 1 2 4 8; do for r in $(echo 0 $((w - 1)) | tr ' ' '\n' | sort -u); do
              timeout -k 10 200 python -u scripts/run_workload.py --config $c --shard $r/$w --repeat 10 \
                >> $O/shards.jsonl 2>> $O/shards.err || fail shards $O/shards.err
            done; done; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "$step done"
done
