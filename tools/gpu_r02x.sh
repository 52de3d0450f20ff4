# Round 2: lsqp4 one-barrier reduce (product) vs the committed two-barrier reduce, and the
# timing probe "next block's rows issued inside phase 2" (measurement build, dbg 128)
set -u
O=gpurun_out/r02x
mkdir -p $O
NEW=$PWD/mpistragglers.jl_amd/_build/libmpiasyncpools.so
OLD=$PWD/mpistragglers.jl_amd/_build_ab/lib_old.so
MEA=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
run() { # label lib dbg
MPA_LIB=$2 MPA_LSQP_DBG=$3 timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/$1.log 2>&1 || exit $?
echo "$1 $(grep rows/ $O/$1.log)"
}
for r in 1 2; do
run old$r $OLD 0
run new$r $NEW 0
run mea0_$r $MEA 0
run dmainp2_$r $MEA 128
done
