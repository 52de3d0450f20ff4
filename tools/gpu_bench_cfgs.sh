# N=1 bench lines of the given configs (default c5 c3 c4) into gpurun_out/cfg_$TAG
set -u
O=gpurun_out/cfg_${TAG:-x}
mkdir -p $O
for c in ${CONFIGS:-c5 c3 c4}; do
timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-20} --warmup 3 > $O/bench_$c.log 2>&1; rc=$?
echo "bench $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
tail -1 $O/bench_$c.log | cut -c1-200
done
