# Round 3, call 5: device-armed worker processes (in-kernel doorbell wait, hip_server.cpp):
# the two-process GPU tests, then N = 2 one-GPU rehearsals of c1 and c2 with the servers
# host-launched (MPA_ARM=0), device-armed where one worker per process (default) and every
# worker device-armed (MPA_ARM=1) (profiles/r03_device_armed.txt)
set -u
O=gpurun_out/r03e
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v -rP --timeout 200 --timeout-method thread > $O/dist.log 2>&1; rc=$?
echo "dist rc=$rc"; grep -E "PASSED|FAILED|passed|failed" $O/dist.log | tail -25; [ $rc -eq 0 ] || exit $rc
for cfg in c1 c2; do
  for arm in 0 2 1; do
    MPA_ARM=$arm MPA_BENCH_ONE_GPU=1 timeout -k 10 240 python -u bench.py --gpus 2 --config $cfg --steps 400 --warmup 50 --no-cpu-baseline > $O/n2_${cfg}_arm$arm.log 2>&1 || exit $?
    grep '^{' $O/n2_${cfg}_arm$arm.log > $O/n2_${cfg}_arm$arm.json; echo "n2 $cfg arm$arm $(python3 -c "import json;d=json.load(open('$O/n2_${cfg}_arm$arm.json'));print(d['value'], d['ms_per_step'])")"
  done
done
