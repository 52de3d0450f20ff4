# Round 2: lsqp4 L2 prefetch with the non-temporal hint (measurement build, MPA_LSQP_DBG bit 4):
# can a longer lead go through the Infinity Cache without thrashing L2?
set -u
O=gpurun_out/r02k
mkdir -p $O
timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/product_pf1.log 2>&1 || exit $?
echo "product pf1 $(grep rows/ $O/product_pf1.log)"
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
for cfg in "1 0" "1 4" "2 4" "4 4" "8 4" "16 4" "4 6" "8 6"; do set -- $cfg
MPA_LSQP_PF=$1 MPA_LSQP_DBG=$2 timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/pf$1_dbg$2.log 2>&1 || exit $?
echo "pf=$1 dbg=$2 $(grep rows/ $O/pf$1_dbg$2.log)"
done
