# Round 2 session 3: workgroups per least-squares launch (MPA_LSQ_GRID) on c3 (fp32, 2048 columns,
# delayed workers launched one task at a time) and c4 (fp64), same box
set -u
O=gpurun_out/r02grid3
mkdir -p $O
for c in c3 c4; do for g in 192 256 384 128; do
MPA_LSQ_GRID=$g timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 > $O/${c}_g$g.log 2>&1 || exit $?
grep '^{' $O/${c}_g$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c grid=$g', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
done; done
