#!/bin/bash
# Round 6: why the one-GPU N = 8 rehearsal (8 processes on GPU 0, c2) runs ~70 it/s while N = 4 runs ~1390: the c2 line
# at N = 5 .. 8 processes on the one GPU (fewer queues per process changed nothing: MPA_OWN_COORD=0, GPU_MAX_HW_QUEUES=1
# gave 64 / 70 it/s, r06q8).
set -u
O=gpurun_out/${1:-r06q8b}; mkdir -p $O
export MPA_BENCH_ONE_GPU=1
for n in 5 6 7 8; do
  timeout -k 10 300 python -u bench.py --gpus $n --config c2 --no-cpu-baseline --steps 100 --warmup 10 > $O/n$n.log 2>&1 || { echo "n$n failed"; tail -5 $O/n$n.log; exit 1; }
  grep '^{' $O/n$n.log | python3 -c "import json,sys;d=json.load(sys.stdin);r=d['roofline'];print('N=$n', d['value'], d['ms_per_step'], 'kernel', r.get('avg_launch_ms'), d.get('placement'))"
done
