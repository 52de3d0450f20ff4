# Round 3, session 2, final tree: the c1 bench command under rocprofv3 --kernel-trace --stats
# (profiles/r03_c1_kernel_stats.csv, r03_c1_timeline_final.txt).
set -u
R=$PWD
O=$R/gpurun_out/r03zx
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c1 -o c1 -- python3 $R/bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline > $O/trace_c1.log 2>&1 || exit $?
echo "trace c1 ok"
