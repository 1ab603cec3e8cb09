#!/bin/bash
# round-2 session c: figure-8 FF deviation with cr_sincos, full GPU suite, clock-stamp placement
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/ff_fig8_deviation.py > gpurun_out/ff_fig8.log 2>&1 || { cat gpurun_out/ff_fig8.log; exit 5; }
cat gpurun_out/ff_fig8.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
QUADTRACK_LIB=build/stamp/libquadtrack.so timeout -k 10 120 python -u scripts/clock_stamp.py --dump gpurun_out/stamps_linear.npz > gpurun_out/clock.log 2>&1 || { cat gpurun_out/clock.log; exit 6; }
cat gpurun_out/clock.log
