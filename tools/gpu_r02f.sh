# Round 2: lsqp4 (one wave per SIMD) — lsqb tests, then isolated launches lsqp4 vs lsqp8 per
# footprint, then c5 bench lsqp4 / lsqp8 / lsqp4
set -u
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lsqb.py -x -v -rP --timeout 180 --timeout-method thread > $O/lsqb_tests.log 2>&1; rc=$?
echo "lsqb tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/lsqb_tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
for v in 4 8; do
MPA_LSQP=$v timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 2048 4096 65536 1048576 > $O/probe_$v.log 2>&1 || exit $?
echo "lsqp$v"; grep rows/ $O/probe_$v.log
done
for v in 4 8 4; do
MPA_LSQP=$v timeout -k 10 240 python -u bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_$v.log 2>&1; rc=$?
echo "c5 lsqp$v rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('$O/c5_$v.log') if l.startswith('{')][-1]);print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'])")"; [ $rc -eq 0 ] || exit $rc
done
