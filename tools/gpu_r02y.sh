# Round 2: lsqp4 strip ring (DMA issued strip by strip inside phase 2, phase 1 waits strip by
# strip) vs the one-barrier row-DMA build and the committed two-barrier build: c5 parity
# tests, then same-box A/B of isolated 8-task launches
set -u
O=gpurun_out/r02y
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lsqb.py -x -v -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
NEW=$PWD/mpistragglers.jl_amd/_build/libmpiasyncpools.so
B1=$PWD/mpistragglers.jl_amd/_build_ab/lib_1bar.so
OLD=$PWD/mpistragglers.jl_amd/_build_ab/lib_old.so
run() { # label lib
MPA_LIB=$2 timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/$1.log 2>&1 || exit $?
echo "$1 $(grep rows/ $O/$1.log)"
}
for r in 1 2; do
run old$r $OLD
run onebar$r $B1
run strip$r $NEW
done
for pf in 0 2; do MPA_LSQP_PF=$pf run strip_pf$pf $NEW; done
