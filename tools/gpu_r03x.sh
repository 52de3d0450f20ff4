# Round 3, session 2: c1 (BASELINE configs[0] shape, latency-bound) on this tree against the
# round-2 final tree (b72e083, built in _bisect/r02 with its own bench.py), same box, 3000 steps
set -u
R=$PWD
O=$R/gpurun_out/r03x
mkdir -p $O
b() {  # label dir
  (cd $2 && timeout -k 10 240 python -u bench.py --config c1 --steps 3000 --warmup 300 --no-cpu-baseline) > $O/$1.log 2>&1 || exit $?
  grep '^{' $O/$1.log > $O/$1.json
  echo "$1 $(python3 -c "import json;d=json.load(open('$O/$1.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'])")"
}
for k in 1 2 3; do
  b r03_$k $R
  b r02_$k $R/_bisect/r02
done
