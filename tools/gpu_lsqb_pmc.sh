# HBM counters of the two c5 passes (8 workers x 262144 rows x 2048 bf16, nwait 8 batches):
# separate FETCH_SIZE / WRITE_SIZE passes over tools/lsqb_mall_probe.py, summarised per kernel.
set -u
R=$PWD
O=$R/gpurun_out/lsqb_pmc_${TAG:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o m -- python3 $R/tools/lsqb_mall_probe.py 262144 > $O/fetch.log 2>&1 || exit $?
echo fetch ok
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o m -- python3 $R/tools/lsqb_mall_probe.py 262144 > $O/write.log 2>&1 || exit $?
echo write ok
cd $R
# one-pass algorithmic bytes of the 8-task batch: A + B + X + G per task
ALG=$(python3 -c "r,c,k=262144,2048,64; print(8*(2*r*c+2*r*k+2*c*k+4*c*k))")
for k in lsqb_resid_kernel lsqb_grad_kernel; do
  python3 tools/pmc_summarize.py --kernel $k --fetch $O/fetch --write $O/write --out $O/$k.json --alg-bytes $ALG --skip 3 || exit $?
done
