# Round 2: lsqp time per block against the A footprint (Infinity-Cache resident vs HBM):
# is the single pass memory- or issue-bound?
set -u
O=gpurun_out/r02e
mkdir -p $O
MPA_LSQP_PF=0 timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 2048 4096 8192 65536 1048576 > $O/probe.log 2>&1 || exit $?
grep rows/ $O/probe.log
# HBM counters of the bench's dominant kernel, c2 and c5, separate FETCH / WRITE passes
R=$PWD
cd /tmp && export TMPDIR=/tmp
for c in c2 c5; do
  st=10; [ $c = c5 ] && st=4
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/${c}_fetch -o m -- python3 $R/bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $R/$O/${c}_fetch.log 2>&1 || exit $?
  echo "$c fetch ok"
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/${c}_write -o m -- python3 $R/bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $R/$O/${c}_write.log 2>&1 || exit $?
  echo "$c write ok"
done
cd $R
python3 tools/pmc_summarize.py --kernel lsq_grad_kernel --fetch $O/c2_fetch --write $O/c2_write --out $O/lsq_pmc_c2.json --alg-bytes 4299227136 --skip 2 || exit $?
C5ALG=$(python3 -c "r,c,k=1048576,2048,64; print(4*(2*r*c+2*r*k+2*c*k+4*c*k))")  # a 1-task and a 7-task launch per epoch: 4 tasks per launch on average
python3 tools/pmc_summarize.py --kernel lsqp_kernel --fetch $O/c5_fetch --write $O/c5_write --out $O/lsq_pmc_c5.json --alg-bytes $C5ALG --skip 4 || exit $?
