# Round 3, session 2: lsqp4 v5 (FULL: phase 2 tail beside the next block's reduce) parity, then a
# same-box c5 A/B against v4 (95d334e) and the round-start library (profiles/r03_c5_full_ab.txt)
set -u
O=gpurun_out/r03s
mkdir -p $O
L=$PWD/mpistragglers.jl_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsqb.py tests/test_gpu_capi_client.py tests/test_gpu_gated.py tests/test_gpu_configs.py -k "lsq or capi or c5 or full or descent" -x -v -rP --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "^(FAILED)|passed|failed|FULL worker" $O/tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
b() {  # label lib
  MPA_LIB=$2 timeout -k 10 240 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/$1.log 2>&1 || exit $?
  grep '^{' $O/$1.log > $O/$1.json
  echo "$1 $(python3 -c "import json;d=json.load(open('$O/$1.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])")"
}
for k in 1 2 3; do
  b v5_$k $L/_build/libmpiasyncpools.so
  b v4_$k $L/_build_ab_v4/libmpiasyncpools.so
  b old$k $L/_build_ab_old/libmpiasyncpools.so
done
