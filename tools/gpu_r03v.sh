# Round 3, session 2: lsqp4 v4 knobs, same box: chunk 0's transposed reads after the barrier
# (RD0_LATE) and the phase-1 read-ahead (AD 2 / 3 / 4); c5 bench lines
set -u
O=gpurun_out/r03v
mkdir -p $O
L=$PWD/mpistragglers.jl_amd
b() {  # label lib
  MPA_LIB=$2 timeout -k 10 240 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/$1.log 2>&1 || exit $?
  grep '^{' $O/$1.log > $O/$1.json
  echo "$1 $(python3 -c "import json;d=json.load(open('$O/$1.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])")"
}
for k in 1 2; do
  b v4_$k $L/_build/libmpiasyncpools.so
  b late_$k $L/_build_ab_late/libmpiasyncpools.so
  b ad4_$k $L/_build_ab_ad4/libmpiasyncpools.so
  b ad2_$k $L/_build_ab_ad2/libmpiasyncpools.so
done
