#!/bin/bash
# kernel A/B: parity suite, bench, clock stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log | cut -c1-400
QUADTRACK_LIB=build/stamp/libquadtrack.so timeout -k 10 120 python -u scripts/clock_stamp.py --seconds 2 --dump gpurun_out/stamps_f.npz > gpurun_out/clock_f.log 2>&1 || { cat gpurun_out/clock_f.log; exit 6; }
cat gpurun_out/clock_f.log
QUADTRACK_LIB=build/stamp/libquadtrack.so timeout -k 10 120 python -u scripts/clock_stamp.py --seconds 2 --motion sinusoidal --ctl lqi > gpurun_out/clock_f_lqi.log 2>&1 || { cat gpurun_out/clock_f_lqi.log; exit 6; }
cat gpurun_out/clock_f_lqi.log
