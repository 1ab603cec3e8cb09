#!/bin/bash
# configs 3-5 on one GPU, each after ~1 s of untimed warm-up; JSON lines to gpurun_out/workloads.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/workloads.jsonl
for c in ${CONFIGS:-3 4 5}; do
  timeout -k 10 300 python -u scripts/run_workload.py --config $c --repeat 10 >> gpurun_out/workloads.jsonl 2> gpurun_out/wl_$c.err || { tail -20 gpurun_out/wl_$c.err; exit 3; }
done
cut -c1-420 gpurun_out/workloads.jsonl
