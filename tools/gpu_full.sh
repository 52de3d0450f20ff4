# Full GPU check of the tree: GPU tests, N=1 bench (c2, with cpu_baseline), c3/c4/c5 benches.
# Run from the repo root on the GPU box:  TAG=r01k bash tools/gpu_full.sh
set -u
T=${TAG:-x}
O=gpurun_out/full_$T
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py > $O/bench_c2.log 2>&1; rc=$?
echo "bench c2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c3 c4 c5}; do
timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-20} --warmup 3 > $O/bench_$c.log 2>&1; rc=$?
echo "bench $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
