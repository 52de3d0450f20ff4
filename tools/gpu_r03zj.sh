# Round 3, session 2: pre-armed launches (c1): the fused-head / pre-arm parity test, then c1
# with pre-arming on / off (MPA_PREARM), alternating, then the c2 line.
set -u
R=$PWD
O=$R/gpurun_out/r03zj
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=30
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "fused_head or timing or descent" > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
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
