# Round 2: column-pair c5 kernel (lsqc_kernel.hip, MPA_LSQP=c): parity against the oracle at
# lookahead 1 and 2, then same-box A/B against the default lsqp4 on isolated 8-task launches
# (tools/lsqb_mall_probe.py)
set -u
O=gpurun_out/r02q
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=20
for la in 1 2; do
MPA_LSQC_LA=$la timeout -k 10 300 python -u -m pytest tests/test_gpu_lsqb.py -m gpu -v -k "lsqc_column_pairs" --timeout 120 --timeout-method thread -s > $O/tests_la$la.log 2>&1; rc=$?
echo "lsqc la=$la tests rc=$rc"; grep -E "rel err|passed|failed|Error" $O/tests_la$la.log | tail -12; [ $rc -eq 0 ] || exit $rc
done
for arm in 4 c1 c2 4 c1 c2; do
  MPA_LSQP=${arm:0:1} MPA_LSQC_LA=${arm:1:1} timeout -k 10 200 python -u tools/lsqb_mall_probe.py 65536 1048576 > $O/probe_$arm.log 2>&1 || { echo "probe $arm failed"; tail -5 $O/probe_$arm.log; exit 1; }
  echo "arm $arm"; grep rows $O/probe_$arm.log
done
