# Round 3, call 9: which part of b343307 slowed the c2 N = 1 launch (0.61 -> 0.73 ms):
# A/B libraries without the device-armed doorbell prologue (ab1), without the tail's remote
# wait and doorbells (ab2), without both (ab3), the head with MPA_TAIL=0, and 1a3da88
set -u
O=gpurun_out/r03i
mkdir -p $O
run() {  # dir label [env]
  (cd $1 && env $3 timeout -k 10 200 python -u bench.py --config c2 --steps 300 --warmup 30 --no-cpu-baseline) > $O/$2.log 2>&1 || exit $?
  grep '^{' $O/$2.log > $O/$2.json
  echo "$2 $(python3 -c "import json;d=json.load(open('$O/$2.json'));print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
}
L=$PWD/mpistragglers.jl_amd
run . head X=1
run . ab1 MPA_LIB=$L/_build_ab1/libmpiasyncpools.so
run . ab2 MPA_LIB=$L/_build_ab2/libmpiasyncpools.so
run . ab3 MPA_LIB=$L/_build_ab3/libmpiasyncpools.so
run . notail MPA_TAIL=0
run _bisect/1a3da88 1a3da88 X=1
