# lsqf timing probes: two-pass baseline, then the fused kernel with the exchange and the B
# loads switched off in turn (MPA_LSQF_DBG; the G it computes is then wrong on purpose)
set -u
O=$PWD/gpurun_out/lsqf_dbg_${TAG:-x}
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=20
timeout -k 10 120 python -u tools/lsqb_mall_probe.py 262144 > $O/two.log 2>&1 || exit $?
for d in ${DBG:-0 1 2}; do
  MPA_LSQF=1 MPA_LSQF_DBG=$d timeout -k 10 120 python -u tools/lsqb_mall_probe.py 262144 > $O/f$d.log 2>&1 || exit $?
done
grep -H pair $O/*.log
