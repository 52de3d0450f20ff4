# lsqq timing probes (MPA_LSQQ_DBG bitmask; the G computed is wrong on purpose)
set -u
O=$PWD/gpurun_out/lsqq_dbg_${TAG:-x}
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=20 MPA_LSQQ=1
for d in ${DBG:-0 1 2 4 8 15}; do
  MPA_LSQQ_DBG=$d timeout -k 10 120 python -u tools/lsqb_mall_probe.py 262144 > $O/d$d.log 2>&1 || exit $?
done
grep -H pair $O/*.log
