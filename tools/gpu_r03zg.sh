# Round 3, session 2: the fused head (the epoch step at the head of the task launch):
# test_gpu.py + the gated replays, then c1 with and without it (MPA_HEAD=0), alternating,
# and the c2 line.
set -u
R=$PWD
O=$R/gpurun_out/r03zg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_gated.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
: > $O/ab.txt
for rep in 1 2 3; do
  for h in 1 0; do
    MPA_HEAD=$h timeout -k 10 120 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/c1_h${h}_$rep.log 2>&1 || exit $?
    python - $O/c1_h${h}_$rep.log $h $rep >> $O/ab.txt <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
x = d.get("exchange") or {}
print("c1_head%s_%s" % (sys.argv[2], sys.argv[3]), d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["launches"], x.get("avg_us"), d["x_norm"])
PY
  done
done
cat $O/ab.txt
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/c2.log 2>&1 || exit $?
grep '^{' $O/c2.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print('c2', d['value'], d['roofline']['frac'], d.get('python_loop_it_per_s'))"
