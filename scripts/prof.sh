#!/bin/bash
# rocprofv3 session for any command: a kernel trace (+ stats), then one PMC pass
# per counter set (each pass its own run, as the counter blocks allow).
#   TAG=name PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU" scripts/prof.sh python3 prog.py args...
# Outputs under gpurun_out/prof_<TAG>/ (trace/ and pmc_<set>/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-run}
mkdir -p $OUT
timeout -k 10 ${PTIMEOUT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- "$@" \
  > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
IFS=';' read -ra SETS <<< "${PMC_SETS:-}"
for PMC in "${SETS[@]}"; do
  [ -z "$PMC" ] && continue
  name=$(echo $PMC | tr ' ' '_')
  timeout -k 10 ${PTIMEOUT:-300} rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc_$name -o run -- "$@" \
    > $OUT/pmc_$name.log 2>&1 || { echo "pmc $PMC failed"; tail -20 $OUT/pmc_$name.log; exit 1; }
done
find $OUT -name "*.csv" | head -50
