# Round 2: lsqp4 in-kernel stamps (measurement build, MPA_LSQP_DBG=64): shader cycles per
# segment of the block loop, per wave, for a sample of workgroups
set -u
O=gpurun_out/r02w
mkdir -p $O
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
for d in 0 64; do
MPA_LSQP_DBG=$d timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/dbg$d.log 2>&1 || exit $?
echo "dbg=$d $(grep rows/ $O/dbg$d.log)"
done
grep -c lsqp4prof $O/dbg64.log
grep lsqp4prof $O/dbg64.log | tail -64 > $O/prof.txt
