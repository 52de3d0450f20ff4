# Round 2: lsqc exchange-ring memory kind A/B (MPA_LSQC_XG: uncached default / fine / coarse)
# against lsqp4, isolated 8-task launches at 2^20 rows per worker, plus the lsqc parity tests
set -u
O=gpurun_out/r02s
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=20
MPA_LSQC_LA=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_lsqb.py -m gpu -v -k "lsqc_column_pairs" --timeout 120 --timeout-method thread -s > $O/tests.log 2>&1; rc=$?
echo "lsqc tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
for arm in 4-x c2-uncached c2-fine c2-coarse c1-uncached c1-coarse 4-x c2-uncached c2-fine c2-coarse; do
  k=${arm%%-*}; xg=${arm#*-}
  MPA_LSQP=${k:0:1} MPA_LSQC_LA=${k:1:1} MPA_LSQC_XG=$xg timeout -k 10 200 python -u tools/lsqb_mall_probe.py 1048576 > $O/ab_$arm.log 2>&1 || { echo "probe $arm failed"; tail -5 $O/ab_$arm.log; exit 1; }
  echo "arm $arm $(grep rows $O/ab_$arm.log)"
done
