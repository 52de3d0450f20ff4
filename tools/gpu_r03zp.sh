# Round 3, session 2: c3 (fp32 2^23 x 2048, 8 workers with Exp(1 ms) delays, nwait 6: mostly
# single-task launches, several overlapping) against the launch grid (measurement build,
# MPA_LSQ_GRID; the product's 192 fills 192 of 256 CUs when a launch runs alone), alternating.
set -u
O=gpurun_out/r03zp
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60
L=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
: > $O/ab.txt
for k in 1 2; do
for g in 192 256 512; do
  MPA_LIB=$L MPA_LSQ_GRID=$g timeout -k 10 200 python -u bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > $O/g${g}_$k.log 2>&1 || exit $?
  echo "grid $g run $k $(grep '^{' $O/g${g}_$k.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])")" | tee -a $O/ab.txt
done; done
