# Round 3, session 2: pre-armed launches released with their predicted step (kPreSame: no mailbox read over
# the bus when the host's step equals the prediction): the tests, then c1 against the
# previous build (_build_ab_prev, MPA_LIB), alternating.
set -u
O=gpurun_out/r03zw
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_gated.py -v --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
P=$PWD/_build_ab_prev/libmpiasyncpools.so
: > $O/ab.txt
for k in 1 2 3; do
for v in new prev; do
  if [ $v = prev ]; then export MPA_LIB=$P; else unset MPA_LIB; fi
  timeout -k 10 120 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/c1_${v}_$k.log 2>&1 || exit $?
  echo "c1 $v run $k $(grep '^{' $O/c1_${v}_$k.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['epoch_steps']['prearmed'], d['epoch_steps'].get('prearm_same'), d['x_norm'])")" | tee -a $O/ab.txt
done; done
