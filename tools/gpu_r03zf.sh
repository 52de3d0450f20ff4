# Round 3, session 2: the sampled-timing test, then the c1 kernel timeline with one launch in
# 16 timed (where the epoch goes once the event cost is off the critical path), and c2 with
# every launch vs one in 8 timed (does the event cost reach the bandwidth-bound config?).
set -u
R=$PWD
O=$R/gpurun_out/r03zf
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "timing or descent" > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
: > $O/c2ab.txt
for rep in 1 2; do
  for tp in 1 8; do
    timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 --no-cpu-baseline --timing-period $tp > $O/c2_${tp}_$rep.log 2>&1 || exit $?
    python - $O/c2_${tp}_$rep.log $tp $rep >> $O/c2ab.txt <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print("c2_tp%s_%s" % (sys.argv[2], sys.argv[3]), d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], d["roofline"]["launches"])
PY
  done
done
cat $O/c2ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c1 -o c1 -- python3 $R/bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/trace_c1.log 2>&1 || exit $?
echo "trace c1 ok"
