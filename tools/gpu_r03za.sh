# Round 3, session 2: bench.py --gpus 2 self-launched with both ranks on GPU 0 (MPA_BENCH_ONE_GPU=1):
# c5 (rank 1 serves workers 5-8 as one batched FULL-form lsqp4 launch), c2, c1
# (profiles/r03_bench_n2_onegpu_*.json)
set -u
O=gpurun_out/r03za
mkdir -p $O
for c in c5 c2 c1; do
  steps=100; [ $c = c5 ] && steps=20; [ $c = c1 ] && steps=2000
  MPA_BENCH_ONE_GPU=1 MPA_WAIT_TIMEOUT_S=60 timeout -k 10 300 python -u bench.py --gpus 2 --config $c --steps $steps --warmup 5 --no-cpu-baseline > $O/n2_$c.log 2>&1 || { tail -5 $O/n2_$c.log; exit 1; }
  grep '^{' $O/n2_$c.log | tail -1 > $O/n2_$c.json
  echo "n2 $c $(python3 -c "import json;d=json.load(open('$O/n2_$c.json'));print(d['value'], d['ms_per_step'], d.get('exchange'))")"
done
