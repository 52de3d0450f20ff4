# N = 8 one-GPU rehearsal of c2: pre-armed single-worker processes (default) vs host-launched (MPA_ARM=0)
set -u
O=gpurun_out/n8arm_${TAG:-x}
mkdir -p $O
for arm in 0 auto 0; do
  if [ $arm = auto ]; then unset MPA_ARM; else export MPA_ARM=$arm; fi
  MPA_BENCH_ONE_GPU=1 MPA_WAIT_TIMEOUT_S=60 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29563 bench.py --gpus 8 --config c2 --steps 100 --warmup 10 > $O/arm_$arm.log 2>&1; rc=$?
  echo "arm=$arm rc=$rc"; grep '^{' $O/arm_$arm.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
