# Round 3, session 2: the shipped c5 tree (lsqp4 v4): bench line, kernel-trace window, and the
# FETCH_SIZE / WRITE_SIZE passes (profiles/r03_bench_c5.json, r03_c5_rocprof_window.json,
# r03_c5_kernel_stats.csv, lsq_pmc_c5.json)
set -u
R=$PWD
O=$R/gpurun_out/r03w
mkdir -p $O
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit $?
grep '^{' $O/bench_c5.log > $O/bench_c5.json; echo bench ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o c5 -- python3 $R/bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_c5.log 2>&1 || exit $?
echo trace ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o c5 -- python3 $R/bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline > $O/fetch.log 2>&1 || exit $?
echo fetch ok
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o c5 -- python3 $R/bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline > $O/write.log 2>&1 || exit $?
echo write ok
cd $R && python3 tools/pmc_summarize.py --fetch $O/fetch --write $O/write --out $O/lsq_pmc_c5.json --kernel lsqp4_kernel --alg-bytes 4429971456 --task-bytes 4429971456
