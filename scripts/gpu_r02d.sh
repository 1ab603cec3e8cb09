#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/ff_fig8_deviation.py > gpurun_out/ff_fig8.log 2>&1 || { cat gpurun_out/ff_fig8.log; exit 5; }
cat gpurun_out/ff_fig8.log
for i in 1 2; do
QUADTRACK_LIB=build/stamp/libquadtrack.so timeout -k 10 120 python -u scripts/clock_stamp.py --seconds 2 --dump gpurun_out/stamps_linear_$i.npz > gpurun_out/clock_$i.log 2>&1 || { cat gpurun_out/clock_$i.log; exit 6; }
done
cat gpurun_out/clock_*.log
