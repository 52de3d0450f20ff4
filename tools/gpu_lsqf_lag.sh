# lsqf: phase-1 lead (MPA_LSQF_LAG) against the no-exchange probe (mode 4) and the real kernel
set -u
O=$PWD/gpurun_out/lsqf_lag_${TAG:-x}
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=20 MPA_LSQF=1
for m in ${MODES:-4 0}; do for l in ${LAGS:-1 2 3 4}; do
  MPA_LSQF_DBG=$m MPA_LSQF_LAG=$l timeout -k 10 120 python -u tools/lsqb_mall_probe.py 262144 > $O/m${m}_l$l.log 2>&1 || exit $?
done; done
grep -H pair $O/*.log
