# Round 3, session 2, final tree: the N-process path at N = 4 and 8 with every rank on GPU 0
# (MPA_BENCH_ONE_GPU=1: host-launched), c2 and c1, so the driver's multi-GPU runs start from a
# path rehearsed on this tree.
set -u
O=gpurun_out/r03zv
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60 MPA_BENCH_ONE_GPU=1
: > $O/lines.txt
for n in 4 8; do
for cfg in c2 c1; do
  st=300; [ $cfg = c1 ] && st=2000
  timeout -k 10 240 python -u bench.py --gpus $n --config $cfg --steps $st --warmup 30 --no-cpu-baseline > $O/${cfg}_n$n.log 2>&1 || { tail -5 $O/${cfg}_n$n.log; exit 1; }
  echo "$cfg N $n $(grep '^{' $O/${cfg}_n$n.log | tail -1 | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['n_gpus'])")" | tee -a $O/lines.txt
done; done
