# c5 iteration: batched-variant parity tests, the c5 bench, a kernel trace of it.
set -u
R=$PWD
T=${TAG:-x}
O=$R/gpurun_out/c5_$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lsqb.py -x -v -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "lsqb tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 3 > $O/bench.log 2>&1 || exit $?
echo bench ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c5 -- python3 $R/bench.py --config c5 --steps 10 --warmup 2 > $O/trace.log 2>&1 || exit $?
echo trace ok
