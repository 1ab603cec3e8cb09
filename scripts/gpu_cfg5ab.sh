#!/bin/bash
# config-5 rollout timing of the in-tree library and of build/ab/<v> builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/cfg5ab.jsonl
for v in tree ${VARS}; do
  lib=lqr-quadcopter-test_amd/quadtrack/_lib/libquadtrack.so
  [ "$v" != tree ] && lib=build/ab/$v/libquadtrack.so
  echo "{\"var\": \"$v\"}" >> gpurun_out/cfg5ab.jsonl
  QUADTRACK_LIB=$(pwd)/$lib timeout -k 10 200 python -u scripts/run_workload.py --config ${CFG:-5} --repeat 8 >> gpurun_out/cfg5ab.jsonl 2>> gpurun_out/cfg5ab.err || exit 3
done
cut -c1-420 gpurun_out/cfg5ab.jsonl
