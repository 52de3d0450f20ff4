# N=2 rehearsal on one GPU, pre-armed servers vs host-launched servers, interleaved.
set -u
T=${TAG:-x}
O=gpurun_out/n2ab_$T
mkdir -p $O
for k in 1 2; do
for arm in 1 0; do
MPA_ARM=$arm MPA_BENCH_ONE_GPU=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2953$k bench.py --gpus 2 > $O/n2_arm${arm}_$k.log 2>&1 || exit $?
echo "arm=$arm run $k ok"
done
done
