# Kernel traces (per-dispatch timestamps + stats) of the c2 and c5 benches, for
# tools/trace_gaps.py and per-pass kernel times; plus the stream wait-value probe.
# Run from the repo root on the GPU box.
set -u
R=$PWD
T=${TAG:-x}
O=$R/gpurun_out/trace_$T
mkdir -p $O
timeout -k 10 60 ./tools/probe_waitvalue > $O/probe_waitvalue.txt 2>&1 || exit $?
echo probe ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o c2 -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/c2.log 2>&1 || exit $?
echo c2 ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/bench.py --config c5 --steps 10 --warmup 2 > $O/c5.log 2>&1 || exit $?
echo c5 ok
cd $R && python3 tools/trace_gaps.py $O/c2 > $O/c2_gaps.json && python3 tools/trace_gaps.py $O/c5 --anchor lsqb_grad_kernel --skip 2 > $O/c5_gaps.json
