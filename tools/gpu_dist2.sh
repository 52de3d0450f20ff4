# GPU suite + N=2 bench rehearsal on one GPU (device path and host-mailbox path).
set -u
O=gpurun_out/d2_${TAG:-x}
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for m in dev host; do
E=""; [ $m = host ] && E="MPA_XGMI=0"
env $E MPA_BENCH_ONE_GPU=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 > $O/n2_$m.log 2>&1; rc=$?
echo "n2 $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
