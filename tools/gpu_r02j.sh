# Round 2: held stale re-dispatches (MPA_HOLD) — full GPU suite, then c5 / c3 / c4 bench A/B
set -u
O=gpurun_out/r02j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/gpu_tests.log | tail -4; [ $rc -eq 0 ] || exit $rc
for h in 1 0 1 0; do
MPA_HOLD=$h timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_hold$h.log 2>&1; rc=$?
echo "c5 hold=$h rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('$O/c5_hold$h.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r['launches'])")"; [ $rc -eq 0 ] || exit $rc
done
for c in c3 c4; do for h in 1 0; do
MPA_HOLD=$h timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > $O/${c}_hold$h.log 2>&1; rc=$?
echo "$c hold=$h rc=$rc $(python3 -c "import json;d=json.loads([l for l in open('$O/${c}_hold$h.log') if l.startswith('{')][-1]);r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r['launches'])")"; [ $rc -eq 0 ] || exit $rc
done; done
