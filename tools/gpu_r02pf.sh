# Round 2 session 3: L2 prefetch lead (MPA_LSQP_PF) re-checked after AD 3 + P2L 1, same box,
# isolated 8-task c5 launches (profiles/r02_c5_strip_ring.txt)
set -u
O=gpurun_out/r02pf
mkdir -p $O
for r in 1 2 3; do for p in 1 2 3 0; do
MPA_LSQP_PF=$p timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/pf$p$r.log 2>&1 || exit $?
echo "pf$p$r $(grep rows/ $O/pf$p$r.log)"
done; done
