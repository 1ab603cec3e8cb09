#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/ff_fig8_deviation.py > gpurun_out/ff_fig8.log 2>&1 || { cat gpurun_out/ff_fig8.log; exit 5; }
cat gpurun_out/ff_fig8.log
PYTEST_ARGS="-x --timeout 300 --timeout-method thread" bash gpu_session.sh
