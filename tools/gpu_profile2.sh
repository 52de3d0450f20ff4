# Round profile set: c2 bench (with cpu_baseline), kernel trace + HBM counters of c2, kernel
# trace of c5.  Run from the repo root on the GPU box:  TAG=r01 bash tools/gpu_profile2.sh
set -u
R=$PWD
O=$R/gpurun_out/prof_${TAG:-x}
mkdir -p $O
timeout -k 10 240 python3 -u bench.py > $O/bench_c2.log 2>&1 || exit $?
echo bench ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c2 -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/trace.log 2>&1 || exit $?
echo trace ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o c2 -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/fetch.log 2>&1 || exit $?
echo fetch ok
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o c2 -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/write.log 2>&1 || exit $?
echo write ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/bench.py --config c5 --steps 10 --warmup 2 > $O/c5.log 2>&1 || exit $?
echo c5 ok
cd $R && python3 tools/pmc_summarize.py --fetch $O/fetch --write $O/write --out $O/lsq_pmc_c2.json --alg-bytes 4299227136 && python3 tools/trace_gaps.py $O/trace > $O/c2_gaps.json
