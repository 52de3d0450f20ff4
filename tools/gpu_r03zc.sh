# Round 3, session 2: c1 kernel timeline on the current tree (rocprofv3 --kernel-trace; profiles/r03_c1_timeline.txt)
set -u
R=$PWD
O=$R/gpurun_out/r03zc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o c1 -- python3 $R/bench.py --config c1 --steps 300 --warmup 30 --no-cpu-baseline > $O/trace.log 2>&1 || exit $?
echo trace ok
