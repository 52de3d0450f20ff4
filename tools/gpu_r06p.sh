#!/bin/bash
# Round 6 checkpoint on the current tree: smoke, the whole -m gpu suite, the default bench line (c2), the
# rocprofv3 kernel traces of the c2 and c5 bench commands with their timed-region windows, and the
# FETCH_SIZE / WRITE_SIZE passes (profiles/r06_*, lsq_pmc_c2.json, lsq_pmc_c5.json).
set -u
R=$PWD
T=${1:-r06p}
O=$R/gpurun_out/$T
mkdir -p $O
KEEP_GOING=1 bash tools/gpu.sh $T smoke tests || exit $?
bash tools/gpu.sh $T bench:c2 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o c2 -- python3 $R/bench.py --config c2 --no-cpu-baseline > $O/trace_c2.log 2>&1 || exit $?
echo "trace c2 ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o c5 -- python3 $R/bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_c5.log 2>&1 || exit $?
echo "trace c5 ok"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c2_fetch -o c2 -- python3 $R/bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/c2_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c2_write -o c2 -- python3 $R/bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/c2_write.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5_fetch -o c5 -- python3 $R/bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline > $O/c5_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5_write -o c5 -- python3 $R/bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline > $O/c5_write.log 2>&1 || exit $?
echo "pmc ok"
cd $R
python3 tools/trace_window.py --trace $O/trace_c2/c2_kernel_trace.csv --bench-log $O/trace_c2.log --kernel lsq_grad_kernel --out $O/r06_c2_rocprof_window.json || exit $?
python3 tools/trace_window.py --trace $O/trace_c5/c5_kernel_trace.csv --bench-log $O/trace_c5.log --kernel lsqp4_kernel --out $O/r06_c5_rocprof_window.json || exit $?
python3 tools/pmc_summarize.py --kernel lsq_grad_kernel --fetch $O/c2_fetch --write $O/c2_write --out $O/lsq_pmc_c2.json --alg-bytes 4299227136 --skip 3 || exit $?
python3 tools/pmc_summarize.py --kernel lsqp4_kernel --fetch $O/c5_fetch --write $O/c5_write --out $O/lsq_pmc_c5.json --alg-bytes 4429971456 --task-bytes 4429971456 --skip 0 || exit $?
echo "all ok"
