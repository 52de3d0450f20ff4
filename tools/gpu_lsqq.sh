# Quad single-pass kernel (MPA_LSQQ=1): single-pass GPU tests, then the probe (8 x 1 GiB)
# against the two passes, with a kernel trace of the quad run
set -u
R=$PWD
O=$R/gpurun_out/lsqq_${TAG:-x}
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=20
timeout -k 10 240 python -u -m pytest tests/test_gpu_lsqb.py -x -v -s -k "single_pass" --timeout 100 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/tests.log | head; exit $rc; }
timeout -k 10 120 python -u tools/lsqb_mall_probe.py 262144 > $O/two.log 2>&1 || exit $?
MPA_LSQQ=1 timeout -k 10 120 python -u tools/lsqb_mall_probe.py 65536 262144 > $O/quad.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
MPA_LSQQ=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o q -- python3 $R/tools/lsqb_mall_probe.py 262144 > $O/trace.log 2>&1 || exit $?
cd $R && grep -h pair $O/two.log $O/quad.log && grep lsqq $O/tr/q_kernel_stats.csv | cut -c1-160
