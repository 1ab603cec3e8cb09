#!/bin/bash
# GPU session for the per-step API and the exact step (run under gpurun):
#   STEPS="tests bench trace pmc exact" TAG=r05a bash scripts/session_step_api.sh
# steps:
#   tests  pytest of the per-step API (tests/test_gpu_batched_env.py; PYTEST_ARGS adds)
#   bench  scripts/step_api_bench.py at 65,536 and 1,048,576 episodes, both modes, LQR and LQI
#   trace  rocprofv3 kernel trace + stats of the bench loop (NS episodes, default 1,048,576 and 65,536; 3,000 steps)
#   pmc    FETCH_SIZE and WRITE_SIZE passes of the same loop (NS episodes, 300 steps)
#   sq     SQ and F64 passes of the closed step at 1,048,576 episodes (VALU / FP64 issue beside HBM)
#   exact  the exact step at 65,536 linear LQR episodes (scripts/flavour_timing.py --cases exact):
#          timing, kernel trace, SQ / SQ2 / F64 passes
# Outputs under gpurun_out/$TAG/.  The first failing step ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-step}
mkdir -p $O
fail() { echo "step $1 failed"; tail -40 "$2"; exit 1; }
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
SQ2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH"
F64="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"
LOOP="scripts/step_api_bench.py --mode closed two_call --ctl lqr lqi"
for step in ${STEPS:-tests bench}; do
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests/test_gpu_batched_env.py -x -v --timeout 300 --timeout-method thread \
             ${PYTEST_ARGS:-} > $O/tests.log 2>&1 || fail tests $O/tests.log
           tail -3 $O/tests.log ;;
    bench) timeout -k 10 600 python -u $LOOP --n ${NS:-65536 1048576} --steps 3000 > $O/step_api.jsonl 2> $O/bench.err \
             || fail bench $O/bench.err
           cat $O/step_api.jsonl ;;
    trace) for n in ${NS:-1048576 65536}; do
             timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$n -o run -- \
               python3 $LOOP --n $n --steps 3000 --warm 20 > $O/trace_$n.log 2>&1 || fail trace $O/trace_$n.log
             cp $(find $O/trace_$n -name "*kernel_stats.csv" | head -1) $O/step_api_kernel_stats_$n.csv
           done ;;
    pmc) for n in ${NS:-1048576 65536}; do
           for P in FETCH_SIZE WRITE_SIZE; do
             timeout -k 10 -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $O/pmc_${P}_$n -o run -- \
               python3 $LOOP --n $n --steps 300 --warm 5 > $O/pmc_${P}_$n.log 2>&1 || fail pmc $O/pmc_${P}_$n.log
             python3 scripts/pmc_summary.py $O/step_api_pmc_${P}_$n.csv \
               $(find $O/pmc_${P}_$n -name "*counter_collection.csv")
           done
         done ;;
    sq) for P in "$SQ" "$F64"; do  # the closed step at 1,048,576 episodes: VALU and FP64 issue
          name=$(echo $P | tr ' ' '_')
          timeout -k 10 -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $O/sq_$name -o run -- \
            python3 scripts/step_api_bench.py --mode closed --ctl lqr --n 1048576 --steps 300 --warm 5 \
            > $O/sq_$name.log 2>&1 || fail sq $O/sq_$name.log
        done
        python3 scripts/pmc_summary.py $O/step_api_pmc_SQ_F64.csv $(find $O/sq_* -name "*counter_collection.csv") ;;
    exact) timeout -k 10 300 python -u scripts/flavour_timing.py --cases exact yaw0 > $O/exact_timing.jsonl 2> $O/exact.err \
             || fail exact $O/exact.err
           timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/exact_trace -o run -- \
             python3 scripts/flavour_timing.py --cases exact --reps 5 > $O/exact_trace.log 2>&1 || fail exact $O/exact_trace.log
           cp $(find $O/exact_trace -name "*kernel_stats.csv" | head -1) $O/exact_kernel_stats.csv
           for PMC in "$SQ" "$SQ2" "$F64"; do
             name=$(echo $PMC | tr ' ' '_')
             timeout -k 10 -s KILL 300 rocprofv3 --pmc $PMC --output-format csv -d $O/exact_pmc_$name -o run -- \
               python3 scripts/flavour_timing.py --cases exact --reps 2 --warmup-s 0 > $O/exact_pmc_$name.log 2>&1 \
               || fail exact $O/exact_pmc_$name.log
           done
           cnt() { find $O/exact_pmc_$(echo $1 | tr ' ' '_') -name "*counter_collection.csv"; }
           python3 scripts/pmc_summary.py $O/exact_pmc_SQ_summary.csv $(cnt "$SQ") $(cnt "$SQ2")
           python3 scripts/pmc_summary.py $O/exact_pmc_F64_summary.csv $(cnt "$F64") ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "$step done"
done
