# Round 2: the c5 single pass (lsqp) — lsqb GPU tests, then c5 bench A/B against the two passes
set -u
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lsqb.py -x -v -rP --timeout 180 --timeout-method thread > $O/lsqb_tests.log 2>&1; rc=$?
echo "lsqb tests rc=$rc"; grep -E "passed|failed|rel err" $O/lsqb_tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
MPA_LSQP=$v timeout -k 10 240 python -u bench.py --config c5 --steps 20 --warmup 3 > $O/c5_lsqp$v.log 2>&1; rc=$?
echo "c5 lsqp=$v rc=$rc $(python3 -c "import json;d=json.loads(open('$O/c5_lsqp$v.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'])")"; [ $rc -eq 0 ] || exit $rc
done
