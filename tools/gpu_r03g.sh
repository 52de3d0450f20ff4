# Round 3, call 7: the cross-process fused tail (rank 0's last local task waits for the remote
# completions and runs the next epoch step, doorbells included), device-armed tasks polling
# their doorbell with relaxed loads, the LDS-DMA helpers with the m0 save / s_nop 0 recipe.
# Two-process GPU tests, the c5 single-pass parity (product and measurement builds), then
# N = 1 and N = 2 one-GPU rehearsals of c1 / c2 (host-launched, default, every worker
# device-armed) and a short c5 bench (profiles/r03_cross_tail.txt)
set -u
O=gpurun_out/r03g
mkdir -p $O
export MPA_WAIT_TIMEOUT_S=60
T="python -u -m pytest -x -v -rP --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_dist.py > $O/dist.log 2>&1; rc=$?
echo "dist rc=$rc"; grep -E "passed|failed" $O/dist.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 $T tests/test_gpu_lsqb.py > $O/lsqb.log 2>&1; rc=$?
echo "lsqb rc=$rc"; grep -E "passed|failed" $O/lsqb.log | tail -3; [ $rc -eq 0 ] || exit $rc
MPA_LIB=mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so timeout -k 10 400 $T tests/test_gpu_lsqb.py -k single_pass > $O/lsqb_measure.log 2>&1; rc=$?
echo "lsqb measure rc=$rc"; grep -E "passed|failed" $O/lsqb_measure.log | tail -3; [ $rc -eq 0 ] || exit $rc
for cfg in c1 c2; do
  timeout -k 10 240 python -u bench.py --config $cfg --steps 400 --warmup 50 --no-cpu-baseline > $O/n1_$cfg.log 2>&1 || exit $?
  grep '^{' $O/n1_$cfg.log > $O/n1_$cfg.json; echo "n1 $cfg $(python3 -c "import json;d=json.load(open('$O/n1_$cfg.json'));print(d['value'], d['ms_per_step'])")"
  for arm in 0 2 1; do
    MPA_ARM=$arm MPA_BENCH_ONE_GPU=1 timeout -k 10 240 python -u bench.py --gpus 2 --config $cfg --steps 400 --warmup 50 --no-cpu-baseline > $O/n2_${cfg}_arm$arm.log 2>&1 || exit $?
    grep '^{' $O/n2_${cfg}_arm$arm.log > $O/n2_${cfg}_arm$arm.json; echo "n2 $cfg arm$arm $(python3 -c "import json;d=json.load(open('$O/n2_${cfg}_arm$arm.json'));print(d['value'], d['ms_per_step'])")"
  done
  MPA_TAIL=0 MPA_BENCH_ONE_GPU=1 timeout -k 10 240 python -u bench.py --gpus 2 --config $cfg --steps 400 --warmup 50 --no-cpu-baseline > $O/n2_${cfg}_notail.log 2>&1 || exit $?
  grep '^{' $O/n2_${cfg}_notail.log > $O/n2_${cfg}_notail.json; echo "n2 $cfg notail $(python3 -c "import json;d=json.load(open('$O/n2_${cfg}_notail.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 || exit $?
grep '^{' $O/c5.log > $O/c5.json; echo "c5 $(python3 -c "import json;d=json.load(open('$O/c5.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])")"
timeout -k 10 120 tools/bin/probe_dma_issue > $O/probe.txt 2>&1 || exit $?
tail -8 $O/probe.txt
