# Round 3, session 2: RB 16 shipped for c1's shape -- the fp64 parity tests and the C client on
# it, then c1 against the launch grid again (measurement build, MPA_LSQ_GRID), alternating.
set -u
O=gpurun_out/r03zn
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -v --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
L=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
: > $O/ab.txt
for k in 1 2; do
for g in 192 96 48 384; do
  MPA_LIB=$L MPA_LSQ_GRID=$g timeout -k 10 120 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/g${g}_$k.log 2>&1 || exit $?
  echo "grid $g run $k $(grep '^{' $O/g${g}_$k.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], d['epoch_steps']['prearmed'])")" | tee -a $O/ab.txt
done; done
