# Round 3, call 1: the gated device replays (tests/test_gpu_gated.py, the gated c1/c3/c4
# configs), then the whole GPU suite
set -u
R=$PWD
O=$R/gpurun_out/r03a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gated.py tests/test_gpu_configs.py -x -v -rP --timeout 180 --timeout-method thread > $O/gated.log 2>&1; rc=$?
echo "gated rc=$rc"; grep -E "^(FAILED)|passed|failed" $O/gated.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "^(FAILED)|passed|failed" $O/gpu_tests.log | tail -3; exit $rc
