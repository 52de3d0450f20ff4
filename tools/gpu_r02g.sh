# Round 2: lsqp4 phase costs (measurement build): full, compute only (no DMA), DMA only
set -u
O=gpurun_out/r02g
mkdir -p $O
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
for d in 0 1 2; do
MPA_LSQP_DBG=$d timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 2048 65536 1048576 > $O/probe_dbg$d.log 2>&1 || exit $?
echo "dbg=$d"; grep rows/ $O/probe_dbg$d.log
done
