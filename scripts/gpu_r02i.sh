#!/bin/bash
# Round-2 measurements at HEAD: configs 3-5 (best of 10 after warm-up), the
# batched DARE kernels, clock stamps of the bench and config-3 loops, and a
# rocprofv3 kernel trace + SQ pass of config 5 (grouped kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/workloads_i.jsonl
for c in 3 4 5; do
  timeout -k 10 300 python -u scripts/run_workload.py --config $c --repeat 10 >> gpurun_out/workloads_i.jsonl 2> gpurun_out/wl_$c.err || { tail -20 gpurun_out/wl_$c.err; exit 3; }
done
timeout -k 10 300 python -u scripts/dare_bench.py > gpurun_out/dare_i.jsonl 2> gpurun_out/dare_i.err || { tail -20 gpurun_out/dare_i.err; exit 4; }
: > gpurun_out/clock_i.jsonl
for mc in "linear lqr" "sinusoidal lqi"; do
  set -- $mc
  QUADTRACK_LIB=$(pwd)/build/stamp/libquadtrack.so timeout -k 10 120 python scripts/clock_stamp.py --motion $1 --ctl $2 \
    --seconds 3 >> gpurun_out/clock_i.jsonl 2>> gpurun_out/clock_i.err || exit 5
done
TAG=r02i CASES="cfg5" bash scripts/profile_workloads.sh > gpurun_out/profw_i.txt 2>&1 || { tail -5 gpurun_out/profw_i.txt; exit 6; }
cut -c1-300 gpurun_out/workloads_i.jsonl gpurun_out/dare_i.jsonl gpurun_out/clock_i.jsonl
