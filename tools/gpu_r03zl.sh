# Round 3, session 2: why c1's launches took 43-52 us in r03zk: c1 under the switches
# (head / pre-arm / deferral), counters and task-launch time, then kernel traces.
set -u
R=$PWD
O=$R/gpurun_out/r03zl
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/c1_$n.log 2>&1 || return $?
  grep '^{' $O/c1_$n.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print('$n', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['launches'], d['epoch_steps'], (d.get('exchange') or {}).get('avg_us'))" | tee -a $O/ab.txt
}
: > $O/ab.txt
run base || exit $?
run nopre MPA_PREARM=0 || exit $?
run nodefer MPA_PREARM=0 MPA_DEFER=0 || exit $?
run nohead MPA_HEAD=0 MPA_DEFER=0 || exit $?
run base2 || exit $?
cd /tmp && export TMPDIR=/tmp
MPA_PREARM=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_nopre -o t -- python3 $R/bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/trace_nopre.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_base -o t -- python3 $R/bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/trace_base.log 2>&1 || exit $?
echo traces ok
