#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log | cut -c1-300
: > gpurun_out/workloads_h.jsonl
for c in 3 5; do
  timeout -k 10 300 python -u scripts/run_workload.py --config $c --repeat 12 >> gpurun_out/workloads_h.jsonl 2> gpurun_out/wl_$c.err || { tail -20 gpurun_out/wl_$c.err; exit 3; }
done
cut -c1-330 gpurun_out/workloads_h.jsonl
