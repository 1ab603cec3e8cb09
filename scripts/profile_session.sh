#!/bin/bash
# rocprofv3 session for the bench workload: kernel trace + stats (the driver's
# bench form, --steps 20 --warmup 5, unless TSTEPS / TWARM say otherwise), then
# separate PMC passes (HBM traffic, VALU instruction mix, issued FP64 VALU
# instructions), each its own run under its own time limit.  Outputs under
# gpurun_out/prof_<tag>/, with the per-kernel condensed CSVs bench.py reads
# (kernel_stats.csv, pmc_FETCH_SIZE.csv, pmc_WRITE_SIZE.csv, pmc_SQ_summary.csv,
# pmc_F64_summary.csv) at its top.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="bench.py --steps ${PSTEPS:-5} --warmup ${PWARM:-1} --warmup-seconds 0 --no-cpu-baseline"
TRACE_BENCH="bench.py --steps ${TSTEPS:-20} --warmup ${TWARM:-5} --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $TRACE_BENCH > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
# EXTRA_PMC: further passes, separated by ';' (counters within a pass by spaces)
IFS=';' read -ra EXTRA <<< "${EXTRA_PMC:-}"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
SQ2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH"
F64="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"
for PMC in "FETCH_SIZE" "WRITE_SIZE" "$SQ" "$SQ2" "$F64" "${EXTRA[@]}"; do
  [ -z "$PMC" ] && continue
  name=$(echo $PMC | tr ' ' '_')
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc_$name -o run -- python3 $BENCH > $OUT/pmc_$name.log 2>&1 || { echo "pmc $PMC failed"; tail -20 $OUT/pmc_$name.log; exit 1; }
done
# condensed per-kernel copies (scripts/pmc_summary.py), the files bench.py reads from profiles/<round>/
cp $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
cnt() { find $OUT/pmc_$1 -name "*counter_collection.csv"; }
python3 scripts/pmc_summary.py $OUT/pmc_FETCH_SIZE.csv $(cnt FETCH_SIZE)
python3 scripts/pmc_summary.py $OUT/pmc_WRITE_SIZE.csv $(cnt WRITE_SIZE)
python3 scripts/pmc_summary.py $OUT/pmc_SQ_summary.csv $(cnt "$(echo $SQ | tr ' ' '_')") $(cnt "$(echo $SQ2 | tr ' ' '_')")
python3 scripts/pmc_summary.py $OUT/pmc_F64_summary.csv $(cnt "$(echo $F64 | tr ' ' '_')")
ls -la $OUT
