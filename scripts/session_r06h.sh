set -o pipefail
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 python -u scripts/group_order_ab.py --shard 0/8 --reps 3 > $O/order_ab.jsonl 2> $O/err.log || exit 1
timeout -k 10 300 python -u scripts/group_order_ab.py --shard 7/8 --reps 2 >> $O/order_ab.jsonl 2>> $O/err.log || exit 1
for v in r05 tree r05 tree; do
  if [ $v = tree ]; then L=$PWD/lqr-quadcopter-test_amd/quadtrack/_lib/libquadtrack.so; else L=$PWD/build/ab/$v/libquadtrack.so; fi
  QUADTRACK_LIB=$L timeout -k 10 200 python scripts/flavour_timing.py --n 1048576 --reps 3 --cases exact exact_rewards \
    | sed "s/^/{\"lib\": \"$v\", \"r\": /; s/$/}/" >> $O/exact_1m.jsonl || exit 1
  QUADTRACK_LIB=$L timeout -k 10 200 python scripts/flavour_timing.py --n 65536 --reps 5 --cases exact yaw0 \
    | sed "s/^/{\"lib\": \"$v\", \"r\": /; s/$/}/" >> $O/exact_64k.jsonl || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; tail -2 $O/tests.log
