# GPU tests, the c2 bench and a probe/bench list given in EXTRA (each step time-limited).
# Run from the repo root on the GPU box:  TAG=x EXTRA="..." bash tools/gpu_check.sh
set -u
T=${TAG:-x}
O=gpurun_out/chk_$T
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py --no-cpu-baseline > $O/bench_c2.log 2>&1; rc=$?
echo "bench c2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-}; do
timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-20} --warmup 3 > $O/bench_$c.log 2>&1; rc=$?
echo "bench $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
