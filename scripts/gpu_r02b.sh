#!/bin/bash
# round-2 session b: new RNG/LQI-gate tests, full GPU suite, figure-8 FF deviation, smoke, bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_rng.py \
  "tests/test_gpu_parity.py::test_lqi_gate_threshold_crossings" > gpurun_out/new_tests.log 2>&1
rc=$?; tail -15 gpurun_out/new_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/ff_fig8_deviation.py > gpurun_out/ff_fig8.log 2>&1 || { cat gpurun_out/ff_fig8.log; exit 5; }
cat gpurun_out/ff_fig8.log
PYTEST_ARGS="-x --timeout 300 --timeout-method thread" bash gpu_session.sh
