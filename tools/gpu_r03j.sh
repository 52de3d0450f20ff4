# Round 3, call 10: the doorbell prologue as a per-launch kernel variant (M_ARMED / ARMED):
# two-process and c5 GPU tests, then c2 / c1 / c5 at N = 1 and the N = 2 one-GPU rehearsals
# with the cross-process fused tail, host-launched (MPA_ARM=0) and device-armed (default)
set -u
O=gpurun_out/r03j
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60
T="python -u -m pytest -x -v -rP --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_dist.py tests/test_gpu_lsqb.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
b() {  # label args...
  local l=$1; shift
  timeout -k 10 240 python -u bench.py "$@" --no-cpu-baseline > $O/$l.log 2>&1 || exit $?
  grep '^{' $O/$l.log > $O/$l.json
  echo "$l $(python3 -c "import json;d=json.load(open('$O/$l.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])")"
}
b n1_c2 --config c2 --steps 400 --warmup 50
b n1_c1 --config c1 --steps 3000 --warmup 300
b n1_c5 --config c5 --steps 20 --warmup 5
export MPA_BENCH_ONE_GPU=1
b n2_c2 --gpus 2 --config c2 --steps 400 --warmup 50
MPA_ARM=0 b n2_c2_arm0 --gpus 2 --config c2 --steps 400 --warmup 50
MPA_TAIL=0 b n2_c2_notail --gpus 2 --config c2 --steps 400 --warmup 50
b n2_c1 --gpus 2 --config c1 --steps 3000 --warmup 300
MPA_ARM=0 b n2_c1_arm0 --gpus 2 --config c1 --steps 3000 --warmup 300
