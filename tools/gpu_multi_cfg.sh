# N=2 rehearsal (both ranks on GPU 0) of every bench config.
set -u
O=gpurun_out/mc_${TAG:-x}
mkdir -p $O
for c in ${CONFIGS:-c2 c5 c3 c4}; do
MPA_BENCH_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 2 --config $c --steps ${STEPS:-20} --warmup 3 > $O/n2_$c.log 2>&1; rc=$?
echo "n2 $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
