#!/bin/bash
# One GPU session: parity tests, smoke, bench.  Each GPU step has its own time
# limit; a crash/timeout (exit >= 2 from pytest, anything nonzero after) stops
# the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log | tail -20; exit 3; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 4; }
tail -3 gpurun_out/bench.log
