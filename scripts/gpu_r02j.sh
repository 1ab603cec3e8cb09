#!/bin/bash
# Round-2 workload numbers at HEAD: configs 3-5 (best of 10 after warm-up) and
# the batched DARE kernels; each GPU step under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/workloads_j.jsonl
for c in 3 4 5; do
  timeout -k 10 300 python -u scripts/run_workload.py --config $c --repeat 10 >> gpurun_out/workloads_j.jsonl 2> gpurun_out/wl_$c.err || { tail -20 gpurun_out/wl_$c.err; exit 3; }
done
timeout -k 10 300 python -u scripts/dare_bench.py > gpurun_out/dare_j.jsonl 2> gpurun_out/dare_j.err || { tail -20 gpurun_out/dare_j.err; exit 4; }
cut -c1-400 gpurun_out/workloads_j.jsonl gpurun_out/dare_j.jsonl
