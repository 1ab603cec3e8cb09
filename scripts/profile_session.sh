#!/bin/bash
# rocprofv3 session for the bench workload: kernel trace + stats, then separate
# PMC passes (HBM traffic, VALU instruction mix).  Outputs under gpurun_out/prof_<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="bench.py --steps ${PSTEPS:-5} --warmup ${PWARM:-1} --warmup-seconds 0 --no-cpu-baseline"
TRACE_BENCH="bench.py --steps ${TSTEPS:-200} --warmup ${TWARM:-20} --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $TRACE_BENCH > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
# EXTRA_PMC: further passes, separated by ';' (counters within a pass by spaces)
IFS=';' read -ra EXTRA <<< "${EXTRA_PMC:-}"
for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH" "${EXTRA[@]}"; do
  [ -z "$PMC" ] && continue
  name=$(echo $PMC | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc_$name -o run -- python3 $BENCH > $OUT/pmc_$name.log 2>&1 || { echo "pmc $PMC failed"; tail -20 $OUT/pmc_$name.log; exit 1; }
done
find $OUT -name "*.csv" | head -50
# condensed copies for profiles/ (per-kernel averages): scripts/pmc_summary.py
