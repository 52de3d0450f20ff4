# Round 2 (session 3, strip-ring lsqp4): full GPU suite, N=1 bench lines (c2 default with the CPU baseline, c5), rocprofv3
# kernel-trace summary and HBM counters of the c5 bench (lsqp4)
set -u
R=$PWD
O=$R/gpurun_out/r02zz
mkdir -p $O
L=$R/mpistragglers.jl_amd
for r in 1 2; do for v in default ad4p1; do
lib=$L/_build/libmpiasyncpools.so; [ $v = ad4p1 ] && lib=$L/_build_ab/lib_ad4p1.so
MPA_LIB=$lib timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/ab_$v$r.log 2>&1 || exit $?
echo "$v $(grep rows/ $O/ab_$v$r.log)"
done; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "^(tests|FAILED)|passed|failed" $O/gpu_tests.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench_c2.log 2>&1 || exit $?
grep '^{' $O/bench_c2.log > $O/bench_n1.json; echo "c2 $(cut -c1-200 $O/bench_n1.json)"
timeout -k 10 400 python -u bench.py --config c5 --steps 30 --warmup 3 > $O/bench_c5.log 2>&1 || exit $?
grep '^{' $O/bench_c5.log > $O/bench_c5.json; echo "c5 $(cut -c1-200 $O/bench_c5.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_trace.log 2>&1 || exit $?
echo c5 trace ok
cd $R && python3 tools/trace_window.py --trace $O/c5/c5_kernel_trace.csv --bench-log $O/c5_trace.log --kernel lsqp4_kernel --out $O/r02_c5_rocprof_window.json || exit $?
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5_fetch -o m -- python3 $R/bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > $O/c5_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5_write -o m -- python3 $R/bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > $O/c5_write.log 2>&1 || exit $?
cd $R
C5ALG=$(python3 -c "r,c,k=1048576,2048,64; print(2*r*c+2*r*k+2*c*k+4*c*k)")  # per task: launches carry 8, 7 or 1 tasks
python3 tools/pmc_summarize.py --kernel lsqp4_kernel --fetch $O/c5_fetch --write $O/c5_write --out $O/lsq_pmc_c5.json --alg-bytes $C5ALG --task-bytes $C5ALG --skip 0 || exit $?
