# GPU round for the batched variant: its parity tests, then the whole GPU suite, then the
# c2 bench and a short c5 bench.  Run from the repo root on the GPU box.
mkdir -p gpurun_out
T=${TAG:-x}
timeout -k 10 300 python -u -m pytest tests/test_gpu_lsqb.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/lsqb_tests_$T.log 2>&1; rc=$?
echo "lsqb tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 240 python -u bench.py > gpurun_out/bench_c2_$T.log 2>&1; rc=$?
echo "bench c2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 3 > gpurun_out/bench_c5_$T.log 2>&1; rc=$?
echo "bench c5 rc=$rc"
exit $rc
