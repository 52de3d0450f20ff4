# Round 3, call 2: gated least-squares replays, the gated c1/c3/c4 configs, the extended C
# client; then the whole GPU suite
set -u
R=$PWD
O=$R/gpurun_out/r03b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gated.py -k lsq tests/test_gpu_configs.py tests/test_gpu_capi_client.py -x -v -rP --timeout 180 --timeout-method thread > $O/focus.log 2>&1; rc=$?
echo "focus rc=$rc"; grep -E "^(FAILED)|passed|failed" $O/focus.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "^(FAILED)|passed|failed" $O/gpu_tests.log | tail -3; exit $rc
