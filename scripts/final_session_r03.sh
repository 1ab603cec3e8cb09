export TMPDIR=/tmp; mkdir -p gpurun_out/r03y
for L in build/ab/h5/libquadtrack.so lqr-quadcopter-test_amd/quadtrack/_lib/libquadtrack.so build/ab/h5/libquadtrack.so lqr-quadcopter-test_amd/quadtrack/_lib/libquadtrack.so; do
  QUADTRACK_LIB=$PWD/$L timeout -k 10 300 python -u scripts/run_workload.py --config 5 --repeat 10 >> gpurun_out/r03y/w5.jsonl || exit 1
done
for T in h5 new; do
  L=build/ab/h5/libquadtrack.so; [ $T = new ] && L=lqr-quadcopter-test_amd/quadtrack/_lib/libquadtrack.so
  QUADTRACK_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r03y/pmc_$T -o run -- python3 scripts/run_workload.py --config 5 --repeat 2 --warmup-s 0 > gpurun_out/r03y/pmc_$T.log 2>&1 || exit 1
done
STEPS="benchab workloads profile" CONFIGS="3" TAG=r03f bash scripts/gpu_session.sh
