# Round 3, session 2, final tree: smoke, the whole -m gpu suite, the c2 line (default bench with
# the CPU baseline), the c1 line (with the MPI CPU baseline), the c5 line, and the kernel traces
# of c2 and c5 (profiles/r03_final2_*, r03_bench_*.json, r03_c2/c5 rocprof windows).
set -u
R=$PWD
O=$R/gpurun_out/r03zr
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "^(FAILED)|passed|failed" $O/gpu_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench_c2.log 2>&1 || exit $?
grep '^{' $O/bench_c2.log > $O/bench_c2.json; echo "c2 $(python3 -c "import json;d=json.load(open('$O/bench_c2.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], d['cpu_baseline']['value'])")"
timeout -k 10 300 python -u bench.py --config c1 --steps 3000 --warmup 300 > $O/bench_c1.log 2>&1 || exit $?
grep '^{' $O/bench_c1.log > $O/bench_c1.json; echo "c1 $(python3 -c "import json;d=json.load(open('$O/bench_c1.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], d['epoch_steps'], (d['cpu_baseline'] or {}).get('value'))")"
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit $?
grep '^{' $O/bench_c5.log > $O/bench_c5.json; echo "c5 $(python3 -c "import json;d=json.load(open('$O/bench_c5.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])")"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o c2 -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/trace_c2.log 2>&1 || exit $?
echo "trace c2 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o c5 -- python3 $R/bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_c5.log 2>&1 || exit $?
echo "trace c5 ok"
