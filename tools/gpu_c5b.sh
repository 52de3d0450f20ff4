# c5 kernel iteration: lsqb GPU tests, per-pass kernel trace of the probe, c5 bench.
set -u
R=$PWD
O=$R/gpurun_out/c5b_${TAG:-x}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lsqb.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o m -- python3 $R/tools/lsqb_mall_probe.py ${SIZES:-8192 262144} > $O/probe.log 2>&1 || exit $?
echo probe ok
cd $R && timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 3 > $O/bench_c5.log 2>&1; rc=$?
echo "bench rc=$rc"; exit $rc
