# Round 3, session 2: the fused head on rank 0 of a multi-process comm (remote workers'
# messages and doorbells from workgroup 0): the distributed and head tests, then c1 / c2 at
# N = 2 on one GPU (MPA_HEAD on / off, armed default) and c1 at N = 1.
set -u
O=gpurun_out/r03zt
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu.py -v --timeout 180 --timeout-method thread -k "dist or two_processes or fused_head or descent" > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
: > $O/ab.txt
for k in 1 2; do
for h in 1 0; do
  MPA_HEAD=$h MPA_BENCH_ONE_GPU=1 MPA_ARM=2 timeout -k 10 180 python -u bench.py --gpus 2 --config c1 --steps 3000 --warmup 100 --no-cpu-baseline > $O/c1n2_h${h}_$k.log 2>&1 || { tail -5 $O/c1n2_h${h}_$k.log; exit 1; }
  echo "c1 N2 head $h run $k $(grep '^{' $O/c1n2_h${h}_$k.log | tail -1 | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")" | tee -a $O/ab.txt
done; done
timeout -k 10 120 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/c1.log 2>&1 || exit $?
grep '^{' $O/c1.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print('c1 N1', d['value'], d['ms_per_step'], d['epoch_steps'])" | tee -a $O/ab.txt
