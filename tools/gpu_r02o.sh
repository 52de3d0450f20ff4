# Round 2: the driver's scaling path rehearsed on one GPU (every rank on GPU 0) after the
# round-2 transport changes: bench.py --gpus N self-launched, N = 2, 4, 8 (c2), N = 2 (c5)
set -u
O=gpurun_out/r02o
mkdir -p $O
for n in 2 4 8; do
MPA_BENCH_ONE_GPU=1 timeout -k 10 300 python -u bench.py --gpus $n --steps 50 --warmup 5 --no-cpu-baseline > $O/c2_n$n.log 2>&1; rc=$?
echo "c2 N=$n rc=$rc $(grep '^{' $O/c2_n$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('exchange'))")"; [ $rc -eq 0 ] || exit $rc
done
MPA_BENCH_ONE_GPU=1 timeout -k 10 400 python -u bench.py --config c5 --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_n2.log 2>&1; rc=$?
echo "c5 N=2 rc=$rc $(grep '^{' $O/c5_n2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"; exit $rc
