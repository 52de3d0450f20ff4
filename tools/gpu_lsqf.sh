# Single-pass c5 kernel (opt-in, MPA_LSQF=1): lsqb GPU tests on the fused kernel (XCD-local
# groups, then every group forced cross-XCD), then the timing probes of tools/gpu_lsqf_dbg.sh;
# every in-kernel wait bounded at 20 s.
set -u
R=$PWD
O=$R/gpurun_out/lsqf_${TAG:-x}
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=20
MPA_LSQF=1 timeout -k 10 240 python -u -m pytest tests/test_gpu_lsqb.py -x -v --timeout 100 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; [ $rc -eq 0 ] || { tail -30 $O/tests.log; exit $rc; }
MPA_LSQF=1 MPA_LSQF_DBG=7 timeout -k 10 240 python -u -m pytest tests/test_gpu_lsqb.py -x -v --timeout 100 --timeout-method thread > $O/tests_mixed.log 2>&1; rc=$?
echo "mixed tests rc=$rc"; [ $rc -eq 0 ] || { tail -30 $O/tests_mixed.log; exit $rc; }
bash tools/gpu_lsqf_dbg.sh
