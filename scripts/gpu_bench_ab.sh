#!/bin/bash
# Bench steadiness check: the driver's short form and the default form in one session.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-benchab}
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20_w5.json 2> $O/bench1.err
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_s100_w20.json 2> $O/bench2.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_s20_w5_b.json 2> $O/bench3.err
python - $O <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["warmup_passes_run"], d["warmup_s"], d["roofline"]["kernel_ms"])
PY
