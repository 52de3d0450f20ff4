# the driver's multi-process launch (torch.distributed.run, one rank per "GPU"), rehearsed with every rank on GPU 0
# (MPA_BENCH_ONE_GPU=1) on the round-5 tree: N = 2 and 4, c2 (the default line) and c5 at N = 2
set -u
O=gpurun_out/r05af
mkdir -p $O
export MPA_BENCH_ONE_GPU=1
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) \
    bench.py --gpus $n --steps 100 --warmup 10 > $O/n$n.log 2>&1 || { echo "N=$n failed"; tail -20 $O/n$n.log; exit 1; }
  grep '^{' $O/n$n.log | python3 -c "import json,sys;d=json.load(sys.stdin);print('N=$n', d['value'], d['ms_per_step'], d.get('exchange'))"
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29610 \
  bench.py --gpus 2 --config c5 --steps 20 --warmup 3 > $O/n2c5.log 2>&1 || { echo "c5 N=2 failed"; tail -20 $O/n2c5.log; exit 1; }
grep '^{' $O/n2c5.log | python3 -c "import json,sys;d=json.load(sys.stdin);print('c5 N=2', d['value'], d['ms_per_step'], d.get('exchange'))"
