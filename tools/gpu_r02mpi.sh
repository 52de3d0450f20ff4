# Round 2 session 3: the MPI transport with GPU worker ranks (tests/test_gpu_mpi.py) on the box
set -u
O=gpurun_out/r02mpi
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_mpi.py -v -s --timeout 150 --timeout-method thread > $O/test.log 2>&1; rc=$?
tail -5 $O/test.log; exit $rc
