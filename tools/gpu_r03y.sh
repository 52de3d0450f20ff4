# Round 3, session 2: final-tree check: smoke, the whole -m gpu suite, the c2 line (default bench
# with the CPU baseline) and the c3 / c4 lines (profiles/r03_final_check.txt, r03_bench_*.json)
set -u
R=$PWD
O=$R/gpurun_out/r03y
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "^(FAILED)|passed|failed" $O/gpu_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench_c2.log 2>&1 || exit $?
grep '^{' $O/bench_c2.log > $O/bench_c2.json; echo "c2 $(python3 -c "import json;d=json.load(open('$O/bench_c2.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])")"
for c in c3 c4; do
  timeout -k 10 400 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit $?
  grep '^{' $O/bench_$c.log > $O/bench_$c.json; echo "$c $(python3 -c "import json;d=json.load(open('$O/bench_$c.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])")"
done
