# Round 2: wide rows (lsqw_kernel.hip) — tests/test_gpu.py
set -u
O=gpurun_out/r02l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/gpu_tests.log | tail -4; exit $rc
