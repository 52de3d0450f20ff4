# Round 3, session 2: where c1's epoch steps run with the fused head on / off (counters), and
# a short kernel trace of each.
set -u
R=$PWD
O=$R/gpurun_out/r03zh
mkdir -p $O
for h in 1 0; do
  MPA_HEAD=$h timeout -k 10 120 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/c1_h$h.log 2>&1 || exit $?
  grep '^{' $O/c1_h$h.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print('head $h', d['value'], d['roofline']['avg_launch_ms'], d['epoch_steps'], d.get('exchange'))"
done
cd /tmp && export TMPDIR=/tmp
MPA_HEAD=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_h1 -o h1 -- python3 $R/bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/trace_h1.log 2>&1 || exit $?
echo "trace ok"
