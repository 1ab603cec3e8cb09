#!/bin/bash
# rocprofv3 kernel trace + SQ counter, issued-FP64 and HBM (FETCH_SIZE, WRITE_SIZE) passes for the
# secondary workloads: config 3 (LQI, sinusoidal), config 4 (per-episode Q/R,
# circular: 262,144 episodes on one GPU, cfg4, and the 65,536-episode shard each
# of its 4 GPUs runs, cfg4s), config 5 (1M episodes, grouped motions, one
# launch; cfg5s: the 131,072-episode shard each of its 8 GPUs runs), and the batched DARE kernels (scripts/dare_bench.py).  Every step is
# time-limited; the first failure ends the script.  Outputs under
# gpurun_out/profw_<tag>/<case>_{trace,sq}/.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/profw_$TAG
mkdir -p $OUT
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
F64="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"
run_case() {  # name, then the python arguments
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${name}_trace -o run -- python3 "$@" \
    > $OUT/${name}_trace.log 2>&1 || { echo "$name trace failed"; tail -20 $OUT/${name}_trace.log; exit 1; }
  local pass=0
  IFS=';' read -ra SETS <<< "${PMC_SETS:-$SQ;FETCH_SIZE;WRITE_SIZE;$F64}"
  for PMC in "${SETS[@]}"; do
    pass=$((pass + 1))
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $PMC --output-format csv -d $OUT/${name}_pmc$pass -o run -- python3 "$@" \
      > $OUT/${name}_pmc$pass.log 2>&1 || { echo "$name pmc $PMC failed"; tail -20 $OUT/${name}_pmc$pass.log; exit 1; }
  done
  echo "$name done"
}
for c in ${CASES:-cfg3 cfg5 dare}; do
  case $c in
    cfg3) run_case cfg3 scripts/run_workload.py --config 3 --repeat 10 ;;
    cfg4) run_case cfg4 scripts/run_workload.py --config 4 --repeat 5 ;;
    cfg4s) run_case cfg4s scripts/run_workload.py --config 4 --episodes 65536 --repeat 10 ;;
    cfg5) run_case cfg5 scripts/run_workload.py --config 5 --repeat 5 ;;
    cfg5s) run_case cfg5s scripts/run_workload.py --config 5 --episodes 131072 --repeat 10 ;;
    dare) run_case dare scripts/dare_bench.py --reps 5 ${DARE_ARGS:-} ;;
  esac
done
