# Round 2 session 3, final tree: full GPU suite, N=1 bench lines (c2 with the CPU baseline,
# c5), rocprofv3 kernel-trace summaries of both benches with their timed-region windows
set -u
R=$PWD
O=$R/gpurun_out/r02end
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "^(FAILED)|passed|failed" $O/gpu_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench_c2.log 2>&1 || exit $?
grep '^{' $O/bench_c2.log > $O/bench_n1.json; echo "c2 $(cut -c1-160 $O/bench_n1.json)"
timeout -k 10 400 python -u bench.py --config c5 --steps 30 --warmup 3 > $O/bench_c5.log 2>&1 || exit $?
grep '^{' $O/bench_c5.log > $O/bench_c5.json; echo "c5 $(cut -c1-160 $O/bench_c5.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o c2 -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_trace.log 2>&1 || exit $?
cd $R
python3 tools/trace_window.py --trace $O/c2/c2_kernel_trace.csv --bench-log $O/c2_trace.log --kernel lsq_grad_kernel --out $O/r02_c2_rocprof_window.json || exit $?
python3 tools/trace_window.py --trace $O/c5/c5_kernel_trace.csv --bench-log $O/c5_trace.log --kernel lsqp4_kernel --out $O/r02_c5_rocprof_window.json || exit $?
