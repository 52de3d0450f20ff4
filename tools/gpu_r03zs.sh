# Round 3, session 2: pre-arming limited to native-only nwait (integer / first_plus): the
# head / pre-arm / descent tests and the c1 line.
set -u
O=gpurun_out/r03zs
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_gated.py -v --timeout 120 --timeout-method thread -k "fused_head or descent or timing or native" > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/c1.log 2>&1 || exit $?
grep '^{' $O/c1.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print('c1', d['value'], d['ms_per_step'], d['epoch_steps'])"
