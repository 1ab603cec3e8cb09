#!/bin/bash
# GPU side of the per-step kernel A/B (profiles/r05/step_kernel_ab.jsonl): the
# libraries scripts/ab_step_build.py built, alternated twice, closed-loop and
# two-call steps at 1,048,576 and 65,536 episodes; then the per-step API and
# trainer tests on the closed-form variant.  Outputs gpurun_out/ab_step/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_step
for r in 1 2; do for v in ${VARIANTS:-head w4 cf cfw3}; do
  QUADTRACK_LIB=$PWD/build/ab_step/$v/libquadtrack.so timeout -k 10 120 python scripts/step_api_bench.py \
    --n 1048576 65536 --steps 1000 --warm 50 --mode closed two_call --ctl lqr \
    | sed "s/^/{\"lib\": \"$v\", \"rep\": $r, \"r\": /; s/$/}/" >> gpurun_out/ab_step/ab.jsonl || exit 1
done; done
QUADTRACK_LIB=$PWD/build/ab_step/cf/libquadtrack.so timeout -k 10 600 python -u -m pytest tests/test_gpu_batched_env.py \
  tests/test_gpu_trainer.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_step/cf_tests.log 2>&1
tail -2 gpurun_out/ab_step/cf_tests.log
