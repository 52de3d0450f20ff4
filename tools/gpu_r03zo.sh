# Round 3, session 2: c1 and c2 at N = 2 with both ranks on GPU 0 (MPA_BENCH_ONE_GPU=1),
# device-armed (MPA_ARM=2, the node's default where a process serves one worker) against
# host-launched (MPA_ARM=0, the rehearsal's default), alternating.
set -u
O=gpurun_out/r03zo
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60 MPA_BENCH_ONE_GPU=1
: > $O/ab.txt
for k in 1 2; do
for cfg in c1 c2; do
for arm in 2 0; do
  st=3000; [ $cfg = c2 ] && st=300
  MPA_ARM=$arm timeout -k 10 180 python -u bench.py --gpus 2 --config $cfg --steps $st --warmup 100 --no-cpu-baseline > $O/${cfg}_a${arm}_$k.log 2>&1 || { tail -5 $O/${cfg}_a${arm}_$k.log; exit 1; }
  echo "$cfg arm $arm run $k $(grep '^{' $O/${cfg}_a${arm}_$k.log | tail -1 | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")" | tee -a $O/ab.txt
done; done; done
