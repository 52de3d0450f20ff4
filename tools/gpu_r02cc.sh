# Round 2 session 3: the C-ABI client (system runtime, exact-size buffers) after the
# out-of-row clamp fix, the MPI + GPU-worker job, then the full GPU suite
set -u
O=gpurun_out/r02cc
mkdir -p $O
timeout -k 10 120 ./mpistragglers.jl_amd/_build/capi_client > $O/capi_client.log 2>&1; rc=$?
cat $O/capi_client.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_mpi.py -v -s --timeout 150 --timeout-method thread > $O/mpi.log 2>&1; rc=$?
grep -E "mpi \+ gpu|passed|failed|Error" $O/mpi.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
grep -E "^(FAILED)|passed|failed" $O/gpu_tests.log | tail -3; exit $rc
