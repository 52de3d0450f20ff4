# Round 2 session 3: lsqp4 phase 2 as 32x32x16 MFMAs (hi and lo share one B operand; half the
# phase-2 instructions), VGPR-form accumulators: c5 parity, C client, same-box A/B vs 16x16x32
set -u
O=gpurun_out/r02m32
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lsqb.py -x -v -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -1; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -10; exit $rc; }
timeout -k 10 120 ./mpistragglers.jl_amd/_build/capi_client > $O/capi.log 2>&1 || { cat $O/capi.log; exit 1; }
grep bf16 $O/capi.log
L=$PWD/mpistragglers.jl_amd
for r in 1 2; do for v in m32 m16; do
lib=$L/_build/libmpiasyncpools.so; [ $v = m16 ] && lib=$L/_build_ab/lib_m16.so
MPA_LIB=$lib timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/ab_$v$r.log 2>&1 || exit $?
echo "$v $(grep rows/ $O/ab_$v$r.log)"
done; done
