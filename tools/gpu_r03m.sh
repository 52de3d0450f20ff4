# Round 3, session 2, call 1 (fresh container): smoke, the whole -m gpu suite, the c2 and c5
# bench lines, and the kernel-trace summaries of both (profiles/r03_final_*).
set -u
R=$PWD
O=$R/gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "^(FAILED)|passed|failed" $O/gpu_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench_c2.log 2>&1 || exit $?
grep '^{' $O/bench_c2.log > $O/bench_c2.json; cat $O/bench_c2.json
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit $?
grep '^{' $O/bench_c5.log > $O/bench_c5.json; cat $O/bench_c5.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o c2 -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/trace_c2.log 2>&1 || exit $?
echo "trace c2 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o c5 -- python3 $R/bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_c5.log 2>&1 || exit $?
echo "trace c5 ok"
