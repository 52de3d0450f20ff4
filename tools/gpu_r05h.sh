set -u
R=$PWD; O=$R/gpurun_out/r05h; mkdir -p $O
bash tools/gpu.sh r05h probe:probe_fg_store || exit $?
ML=$R/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
for v in wave kernel; do
  if [ $v = kernel ]; then EXTRA="MPA_ARM_WAIT=kernel MPA_ARM_WAIT_FORCE=1"; else EXTRA=""; fi
  (cd /tmp && env MPA_LIB=$ML $EXTRA MPA_WAIT_TIMEOUT_S=60 MPA_BENCH_ONE_GPU=1 MPA_BENCH_ROWS=65536 MPA_BENCH_PLACEMENT=0,0,0,0,0,0,0,1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$v -o %pid% -- python3 $R/bench.py --gpus 2 --config c2 --no-cpu-baseline --steps 2000 --warmup 100 > $O/trace_$v.log 2>&1) || { echo "trace $v failed"; tail -5 $O/trace_$v.log; exit 1; }
  grep '^{' $O/trace_$v.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['ms_per_step'])"
done
