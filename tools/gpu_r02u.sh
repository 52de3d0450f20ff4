# Round 2: lsqp4 with the DMA ON and parts of the compute removed (measurement build):
# does the 8-task launch follow C (compute per block) or the DMA latency?
set -u
O=gpurun_out/r02u
mkdir -p $O
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
for d in 0 16 8 32 48 56 2; do
MPA_LSQP_DBG=$d timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/dbg$d.log 2>&1 || exit $?
echo "dbg=$d $(grep rows/ $O/dbg$d.log)"
done
