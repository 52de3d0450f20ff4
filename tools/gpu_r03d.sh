# Round 3, call 4: LDS-DMA ingest per CU by where the bytes live (HBM / Infinity Cache / L2;
# profiles/r03_dma_issue_probe.txt), the device-buffer check, the c1 bench line with the MPI
# CPU baseline (profiles/r03_bench_c1.json), and the N = 2 one-GPU rehearsals of c1 and c2
# before the control-path work (profiles/r03_n2_onegpu_before.txt)
set -u
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 180 tools/bin/probe_dma_issue > $O/probe.txt 2>&1; rc=$?
tail -30 $O/probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -k "host_buffers" -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c1 --steps 3000 --warmup 300 --cpu-seconds 10 > $O/bench_c1.log 2>&1 || exit $?
grep '^{' $O/bench_c1.log > $O/bench_c1.json; cut -c1-300 $O/bench_c1.json
for cfg in c1 c2; do
  MPA_BENCH_ONE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --config $cfg --steps 400 --warmup 50 --no-cpu-baseline > $O/n2_$cfg.log 2>&1 || exit $?
  grep '^{' $O/n2_$cfg.log > $O/n2_$cfg.json; echo "n2 $cfg $(cut -c1-200 $O/n2_$cfg.json)"
done
