# Round 3, session 2: lsqp4 v3 timing probes (measurement builds, wrong results; -DMPA_LSQP4_PROBE):
# 1 no strip DMAs in the block loop, 2 no cross-wave exchange / barrier, 4 no phase-1 MFMAs,
# 3 = 1 + 2; same box (profiles/r03_c5_probes.txt)
set -u
O=gpurun_out/r03q
mkdir -p $O
L=$PWD/mpistragglers.jl_amd
b() {  # label lib
  MPA_LIB=$2 timeout -k 10 240 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/$1.log 2>&1 || exit $?
  grep '^{' $O/$1.log > $O/$1.json
  echo "$1 $(python3 -c "import json;d=json.load(open('$O/$1.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])")"
}
for k in 1 2; do
  b base$k $L/_build/libmpiasyncpools.so
  b nodma$k $L/_build_ab_p1/libmpiasyncpools.so
  b noxchg$k $L/_build_ab_p2/libmpiasyncpools.so
  b nop1mfma$k $L/_build_ab_p4/libmpiasyncpools.so
  b nodma_noxchg$k $L/_build_ab_p3/libmpiasyncpools.so
done
