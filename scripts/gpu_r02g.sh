#!/bin/bash
# round-2 profile set r02b at the one-compare vote kernel: workloads 3-5 timings,
# bench-kernel trace + PMC passes, config 3 / 5 / DARE traces + SQ counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/workloads_r02b.jsonl
for c in 3 4 5; do
  timeout -k 10 300 python -u scripts/run_workload.py --config $c --repeat 5 >> gpurun_out/workloads_r02b.jsonl 2> gpurun_out/wl_$c.err || { tail -20 gpurun_out/wl_$c.err; exit 3; }
done
cut -c1-300 gpurun_out/workloads_r02b.jsonl
TAG=r02b bash scripts/profile_session.sh || exit 4
TAG=r02b bash scripts/profile_workloads.sh || exit 5
