# Multi-process path on one GPU: the dist GPU tests, then the N=2 bench rehearsal (both
# ranks on GPU 0) and the N=1 bench for comparison.  Run from the repo root on the GPU box.
set -u
T=${TAG:-x}
O=gpurun_out/dist_$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "dist tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
MPA_BENCH_ONE_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 > $O/bench_n2.log 2>&1; rc=$?
echo "bench n2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py --no-cpu-baseline > $O/bench_n1.log 2>&1; rc=$?
echo "bench n1 rc=$rc"; exit $rc
