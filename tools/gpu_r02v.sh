# Round 2: lsqp4 one-barrier reduce (lane swaps, -B folded into wave 0) vs the two-barrier
# reduce: c5 parity tests, then same-box A/B of isolated 8-task launches
set -u
O=gpurun_out/r02v
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lsqb.py -x -v -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
NEW=$PWD/mpistragglers.jl_amd/_build/libmpiasyncpools.so
OLD=$PWD/mpistragglers.jl_amd/_build_ab/lib_old.so
for r in 1 2; do
for v in OLD NEW; do
eval L=\$$v
MPA_LIB=$L timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/$v$r.log 2>&1 || exit $?
echo "$v $(grep rows/ $O/$v$r.log)"
done
done
