# Round 3, session 2: c1 (3 fp64 workers of 4096 x 64, nwait 2; latency-bound) against the lsq
# launch grid (measurement build, MPA_LSQ_GRID = workgroups per launch, split over the tasks)
# (profiles/r03_c1_grid.txt)
set -u
O=gpurun_out/r03zb
mkdir -p $O
L=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
for k in 1 2; do
for g in ${GRIDS:-192 96 48 24 12}; do
  MPA_LIB=$L MPA_LSQ_GRID=$g timeout -k 10 120 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/g${g}_$k.log 2>&1 || exit $?
  echo "grid $g run $k $(grep '^{' $O/g${g}_$k.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'])")"
done; done
