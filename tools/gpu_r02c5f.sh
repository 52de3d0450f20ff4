# Round 2 session 3, lsqp4 with AD 3 / P2L 1 shipped: c5 parity (bf16 tests, C client), c5 bench line,
# rocprofv3 kernel trace over the timed region, HBM counters (profiles/r02_bench_c5.json,
# r02_c5_rocprof_window.json, r02_c5_kernel_stats.csv, lsq_pmc_c5.json)
set -u
R=$PWD
O=$R/gpurun_out/r02c5f
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_lsqb.py tests/test_gpu_capi_client.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --config c5 --steps 30 --warmup 3 > $O/bench_c5.log 2>&1 || exit $?
grep '^{' $O/bench_c5.log > $O/bench_c5.json; echo "c5 $(cut -c1-160 $O/bench_c5.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_trace.log 2>&1 || exit $?
cd $R && python3 tools/trace_window.py --trace $O/c5/c5_kernel_trace.csv --bench-log $O/c5_trace.log --kernel lsqp4_kernel --out $O/r02_c5_rocprof_window.json || exit $?
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5_fetch -o m -- python3 $R/bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > $O/c5_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5_write -o m -- python3 $R/bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > $O/c5_write.log 2>&1 || exit $?
cd $R
C5ALG=$(python3 -c "r,c,k=1048576,2048,64; print(2*r*c+2*r*k+2*c*k+4*c*k)")  # per task: launches carry 8, 7 or 1 tasks
python3 tools/pmc_summarize.py --kernel lsqp4_kernel --fetch $O/c5_fetch --write $O/c5_write --out $O/lsq_pmc_c5.json --alg-bytes $C5ALG --task-bytes $C5ALG --skip 0 || exit $?
