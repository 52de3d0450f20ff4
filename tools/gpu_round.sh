mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_${TAG:-x}.log 2>&1; rc=$?
echo "tests rc=$rc"; ok $rc || exit $rc
timeout -k 10 240 python -u bench.py > gpurun_out/bench_${TAG:-x}.log 2>&1; rc=$?
echo "bench rc=$rc"; ok $rc || exit $rc
MPA_BENCH_ONE_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 > gpurun_out/bench_${TAG:-x}_n2.log 2>&1; rc=$?
echo "bench2 rc=$rc"
exit $rc
