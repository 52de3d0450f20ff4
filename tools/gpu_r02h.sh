# Round 2: lsqp4 with cheaper DMA addressing and the L2 prefetch lead: tests, lead sweep,
# phase costs (measurement build)
set -u
O=gpurun_out/r02h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lsqb.py -x -v -rP --timeout 180 --timeout-method thread -k "lsqp4 or vs_oracle or c5_shard or counters or stragglers" > $O/lsqb_tests.log 2>&1; rc=$?
echo "lsqb tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/lsqb_tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
for pf in 0 1 2 3 4; do
MPA_LSQP_PF=$pf timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 65536 1048576 > $O/probe_pf$pf.log 2>&1 || exit $?
echo "pf=$pf"; grep rows/ $O/probe_pf$pf.log
done
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
for d in 1 2; do
MPA_LSQP_DBG=$d timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 65536 1048576 > $O/probe_dbg$d.log 2>&1 || exit $?
echo "dbg=$d"; grep rows/ $O/probe_dbg$d.log
done
MPA_LSQP_PF=2 MPA_LSQP_DBG=2 timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 65536 1048576 > $O/probe_dbg2pf2.log 2>&1 || exit $?
echo "dbg=2 pf=2"; grep rows/ $O/probe_dbg2pf2.log
