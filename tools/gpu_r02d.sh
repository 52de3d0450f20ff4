# Round 2: lsqp L2 prefetch lead (MPA_LSQP_PF) and per-worker grid share (MPA_LSQP_SHARE):
# lsqb tests, isolated 8-task launches per lead, c5 bench share on / off
set -u
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lsqb.py -x -v -rP --timeout 180 --timeout-method thread > $O/lsqb_tests.log 2>&1; rc=$?
echo "lsqb tests rc=$rc"; grep -E "passed|failed" $O/lsqb_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
for pf in 0 1 2 3 4 6; do
MPA_LSQP_PF=$pf timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/probe_pf$pf.log 2>&1 || exit $?
echo "pf=$pf $(grep rows/ $O/probe_pf$pf.log)"
done
for sh in 1 0; do
MPA_LSQP_SHARE=$sh timeout -k 10 240 python -u bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_share$sh.log 2>&1; rc=$?
echo "c5 share=$sh rc=$rc $(python3 -c "import json;d=json.loads(open('$O/c5_share$sh.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'],d['roofline']['launches'])")"; [ $rc -eq 0 ] || exit $rc
done
