# Round 3, session 2: lsqp4 pipelined tail size (MPA_LSQP4_HC = head chunks: 5, 6, 7) against
# v4 and the same tree without the pipeline (PIPE=0, = v4's loop); same box, c5 bench lines
set -u
O=gpurun_out/r03t
mkdir -p $O
L=$PWD/mpistragglers.jl_amd
b() {  # label lib
  MPA_LIB=$2 timeout -k 10 240 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/$1.log 2>&1 || exit $?
  grep '^{' $O/$1.log > $O/$1.json
  echo "$1 $(python3 -c "import json;d=json.load(open('$O/$1.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])")"
}
for k in 1 2; do
  b hc5_$k $L/_build/libmpiasyncpools.so
  b hc6_$k $L/_build_ab_hc6/libmpiasyncpools.so
  b hc7_$k $L/_build_ab_hc7/libmpiasyncpools.so
  b nopipe_$k $L/_build_ab_nopipe/libmpiasyncpools.so
  b v4_$k $L/_build_ab_v4/libmpiasyncpools.so
done
