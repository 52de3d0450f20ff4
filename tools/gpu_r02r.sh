# Round 2: lsqc phase probes (measurement build: MPA_LSQP_DBG 1 no A DMA, 2 no exchange,
# 8 / 32 no phase-1 / phase-2 MFMAs), isolated 8-task launches at 2^20 rows per worker
set -u
O=gpurun_out/r02r
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=20 MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so MPA_LSQP=c
for la in 1 2; do
for dbg in 0 2 40 42; do
  MPA_LSQC_LA=$la MPA_LSQP_DBG=$dbg timeout -k 10 120 python -u tools/lsqb_mall_probe.py 1048576 > $O/p_${la}_$dbg.log 2>&1 || { echo "probe la=$la dbg=$dbg failed"; tail -5 $O/p_${la}_$dbg.log; exit 1; }
  echo "la=$la dbg=$dbg $(grep rows $O/p_${la}_$dbg.log)"
done
done
unset MPA_LIB MPA_LSQP
for arm in 4 c1 c2 4 c1 c2; do
  MPA_LSQP=${arm:0:1} MPA_LSQC_LA=${arm:1:1} timeout -k 10 200 python -u tools/lsqb_mall_probe.py 1048576 > $O/ab_$arm.log 2>&1 || { echo "probe $arm failed"; tail -5 $O/ab_$arm.log; exit 1; }
  echo "arm $arm $(grep rows $O/ab_$arm.log)"
done
