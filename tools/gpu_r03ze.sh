# Round 3, session 2: c1 (latency-bound) with the HIP timing events on every launch, on one in
# 16, and effectively off (one in 10^6), alternating on one box, 3000 epochs each.
set -u
R=$PWD
O=$R/gpurun_out/r03ze
mkdir -p $O
: > $O/ab.txt
for rep in 1 2 3; do
  for tp in 1 16 1000000; do
    timeout -k 10 120 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline --timing-period $tp > $O/c1_${tp}_$rep.log 2>&1 || exit $?
    python - $O/c1_${tp}_$rep.log $tp $rep >> $O/ab.txt <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
x = d.get("exchange") or {}
print("tp%s_%s" % (sys.argv[2], sys.argv[3]), d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["launches"], x.get("avg_us"))
PY
  done
done
cat $O/ab.txt
