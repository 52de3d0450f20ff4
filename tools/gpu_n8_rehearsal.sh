# N = 4 and N = 8 rehearsal of the bench (every rank on GPU 0): at N = 8 each process serves
# ONE worker, the pre-armed path the driver's 8-GPU run takes
set -u
O=gpurun_out/n8_${TAG:-x}
mkdir -p $O
for n in ${NS:-4 8}; do
for c in ${CONFIGS:-c2}; do
MPA_BENCH_ONE_GPU=1 MPA_WAIT_TIMEOUT_S=60 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus $n --config $c --steps ${STEPS:-50} --warmup 5 > $O/n${n}_$c.log 2>&1; rc=$?
echo "n$n $c rc=$rc"; tail -1 $O/n${n}_$c.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
done; done
