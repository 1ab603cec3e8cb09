#!/bin/bash
# Rebuild the HIP library from source on the GPU box (run under gpurun), so
# that the tests that follow load a library built there, not the one pushed:
#   TAG=r05n bash scripts/box_build.sh && STEPS="tests smoke" TAG=r05n bash scripts/gpu_session.sh
# Writes gpurun_out/$TAG/box_build.log (make output, the built files, the
# library's sha256).  A heartbeat line every 30 s keeps the call from looking
# hung while the longest translation unit compiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-build}
mkdir -p $O
LOG=$O/box_build.log
(while sleep 30; do echo "build running $(date +%T)"; done) &
HB=$!
start=$(date +%s)
timeout -k 10 900 make -C lqr-quadcopter-test_amd -B -j16 > $LOG 2>&1
rc=$?
kill $HB
echo "make rc=$rc in $(( $(date +%s) - start )) s" | tee -a $LOG
[ $rc -eq 0 ] || { tail -30 $LOG; exit 1; }
ls -la --time-style=full-iso lqr-quadcopter-test_amd/quadtrack/_lib/ >> $LOG
sha256sum lqr-quadcopter-test_amd/quadtrack/_lib/libquadtrack.so | tee -a $LOG
