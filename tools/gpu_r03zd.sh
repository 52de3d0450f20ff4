# Round 3, session 2: c1 host + kernel timeline (rocprofv3 --kernel-trace --hip-trace, no counters)
# to see where the ~43 us epoch goes between the two kernels (profiles/r03_c1_timeline.txt)
set -u
R=$PWD
O=$R/gpurun_out/r03zd
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/trace -o c1 -- python3 $R/bench.py --config c1 --steps 200 --warmup 20 --no-cpu-baseline > $O/trace.log 2>&1 || exit $?
echo trace ok
ls $O/trace
