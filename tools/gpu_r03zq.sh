# Round 3, session 2: c2 with every launch timed vs one in 8 (--timing-period), at N = 1 and
# at N = 2 on one GPU, alternating on one box.
set -u
O=gpurun_out/r03zq
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60
: > $O/ab.txt
for k in 1 2 3; do
for tp in 1 8; do
  timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 --no-cpu-baseline --timing-period $tp > $O/n1_tp${tp}_$k.log 2>&1 || exit $?
  echo "N1 tp $tp run $k $(grep '^{' $O/n1_tp${tp}_$k.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['launches'])")" | tee -a $O/ab.txt
done; done
for k in 1 2; do
for tp in 1 8; do
  MPA_BENCH_ONE_GPU=1 timeout -k 10 200 python -u bench.py --gpus 2 --steps 300 --warmup 30 --no-cpu-baseline --timing-period $tp > $O/n2_tp${tp}_$k.log 2>&1 || exit $?
  echo "N2 tp $tp run $k $(grep '^{' $O/n2_tp${tp}_$k.log | tail -1 | python3 -c "import sys,json;d=json.loads(sys.stdin.read());r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['launches'])")" | tee -a $O/ab.txt
done; done
