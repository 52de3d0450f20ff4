# Same-box A/B of the least-squares launch grid (MPA_LSQ_GRID, workgroups per launch) on the
# c2 / c3 / c4 benches, alternating: the in-tree default vs ${GRID_B:-192}.
set -u
O=gpurun_out/grid_${TAG:-x}
mkdir -p $O
for k in 1 2; do
  for c in ${CONFIGS:-c2 c3 c4}; do
    for g in ${GRID_A:-512} ${GRID_B:-192}; do
      MPA_LSQ_GRID=$g timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline > $O/${c}_g${g}_$k.log 2>&1 || exit $?
      echo "$c grid $g round $k: $(tail -1 $O/${c}_g${g}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["achieved"], r["frac"])')"
    done
  done
done
