#!/bin/bash
# Round-6 A/B of the per-step kernel by kernel time (after the host-side
# trim the 65,536-episode step is GPU-bound): head vs cf
# (scripts/ab_step_build.py) closed steps, rocprofv3 kernel trace of each,
# alternated twice, at NS episodes (default 65,536 and 262,144).
# Outputs gpurun_out/ab_step6/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ab_step6
mkdir -p $O
for r in 1 2; do for v in ${VARIANTS:-head cf}; do for n in ${NS:-65536 262144}; do
  QUADTRACK_LIB=$PWD/build/ab_step/$v/libquadtrack.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $O/t_${v}_${n}_$r -o run -- python3 scripts/step_api_bench.py --mode closed --ctl lqr \
    --n $n --steps 2000 --warm 50 > $O/t_${v}_${n}_$r.log 2>&1 || { tail -20 $O/t_${v}_${n}_$r.log; exit 1; }
  f=$(find $O/t_${v}_${n}_$r -name "*kernel_stats.csv" | head -1)
  avg=$(grep closed_step_kernel $f | awk -F'","' '{print $4}')
  wall=$(grep -o '"ms_per_step": [0-9.e-]*' $O/t_${v}_${n}_$r.log | awk '{print $2}')
  echo "{\"lib\": \"$v\", \"rep\": $r, \"n\": $n, \"kernel_avg_ns\": $avg, \"ms_per_step\": $wall}" | tee -a $O/ab.jsonl
done; done; done
