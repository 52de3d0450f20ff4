# Round 3, session 2: c1's task kernel, rows per wave iteration 4 (shipped) / 8 / 16 (measurement
# build, MPA_LSQ_SMALL_RB), alternating on one box, 3000 epochs each.
set -u
O=gpurun_out/r03zm
mkdir -p $O
L=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
: > $O/ab.txt
for k in 1 2; do
for rb in 4 8 16; do
  MPA_LIB=$L MPA_LSQ_SMALL_RB=$rb timeout -k 10 120 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/rb${rb}_$k.log 2>&1 || exit $?
  echo "rb $rb run $k $(grep '^{' $O/rb${rb}_$k.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], d['epoch_steps']['prearmed'], d['x_norm'])")" | tee -a $O/ab.txt
done; done
