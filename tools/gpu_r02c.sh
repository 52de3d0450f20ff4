# Round 2: c5 lsqp in isolation (one 8-task launch per epoch, nwait 8) at the c5 shard size,
# HBM counters of lsqp_kernel, then rocprofv3 kernel-trace summaries of bench c2 and c5.
set -u
R=$PWD
O=$R/gpurun_out/r02c
mkdir -p $O
MPA_LSQP=1 timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 262144 1048576 > $O/probe_lsqp.log 2>&1 || exit $?
cat $O/probe_lsqp.log | grep rows/
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o m -- python3 $R/tools/lsqb_mall_probe.py 262144 > $O/fetch.log 2>&1 || exit $?
echo fetch ok
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o m -- python3 $R/tools/lsqb_mall_probe.py 262144 > $O/write.log 2>&1 || exit $?
echo write ok
cd $R
ALG=$(python3 -c "r,c,k=262144,2048,64; print(8*(2*r*c+2*r*k+2*c*k+4*c*k))")
python3 tools/pmc_summarize.py --kernel lsqp_kernel --fetch $O/fetch --write $O/write --out $O/lsqp_pmc_probe.json --alg-bytes $ALG --skip 3 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5.log 2>&1 || exit $?
echo c5 trace ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o c2 -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/c2.log 2>&1 || exit $?
echo c2 trace ok
