# Round 2: strip-ring lsqp4 variants (same box): phase-1 read-ahead AD 8 (product) / 6 / 4,
# phase-2 read lookahead 2 chunks
set -u
O=gpurun_out/r02z
mkdir -p $O
L=$PWD/mpistragglers.jl_amd
run() { # label lib
MPA_LIB=$2 timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/$1.log 2>&1 || exit $?
echo "$1 $(grep rows/ $O/$1.log)"
}
for r in 1 2; do
run ad8_$r $L/_build/libmpiasyncpools.so
run ad6_$r $L/_build_ab/lib_ad6.so
run ad4_$r $L/_build_ab/lib_ad4.so
run p2l2_$r $L/_build_ab/lib_p2l2.so
done
