# Round 3, session 2: held stale re-dispatches deferred into the next epoch step + pre-armed
# launches: the whole -m gpu suite, c1 with pre-arming on / off alternating, c2 and c5 lines.
set -u
R=$PWD
O=$R/gpurun_out/r03zk
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/gpu_tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -20; exit $rc; }
: > $O/ab.txt
for rep in 1 2 3; do
  for p in 1 0; do
    MPA_PREARM=$p timeout -k 10 120 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/c1_p${p}_$rep.log 2>&1 || exit $?
    grep '^{' $O/c1_p${p}_$rep.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print('c1_prearm$p', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['launches'], d['epoch_steps'], d['x_norm'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/c2.log 2>&1 || exit $?
grep '^{' $O/c2.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print('c2', d['value'], d['roofline']['frac'], d.get('python_loop_it_per_s'))"
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 || exit $?
grep '^{' $O/c5.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print('c5', d['value'], d['roofline']['frac'], d['epoch_steps'])"
