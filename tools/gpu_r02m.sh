# Round 2: lsqp4 compute breakdown (measurement build, no DMA): which phase costs what
set -u
O=gpurun_out/r02m
mkdir -p $O
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
for d in 0 1 9 17 33 41 49 25 57; do
MPA_LSQP_DBG=$d timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/dbg$d.log 2>&1 || exit $?
echo "dbg=$d $(grep rows/ $O/dbg$d.log)"
done
