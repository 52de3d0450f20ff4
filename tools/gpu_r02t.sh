# Round 2: lsqc probes (measurement build): 256 = block DMAs issued after barrier C instead of A
# (the exchange's stores / polls then do not queue behind them), at lookahead 1 and 2; 2 = no
# exchange; against lsqp4 (product build)
set -u
O=gpurun_out/r02t
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=20 MPA_LSQP=c
for arm in 2-0 2-256 1-256 2-2 1-0; do
  MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so MPA_LSQC_LA=${arm%%-*} MPA_LSQP_DBG=${arm#*-} timeout -k 10 120 python -u tools/lsqb_mall_probe.py 1048576 > $O/p_$arm.log 2>&1 || { echo "probe $arm failed"; tail -5 $O/p_$arm.log; exit 1; }
  echo "la-dbg=$arm $(grep rows $O/p_$arm.log)"
done
MPA_LSQP=4 timeout -k 10 120 python -u tools/lsqb_mall_probe.py 1048576 > $O/p_lsqp4.log 2>&1 || exit 1
echo "lsqp4 $(grep rows $O/p_lsqp4.log)"
