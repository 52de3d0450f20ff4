#!/bin/bash
# Round 6: the driver's N = 2 / 4 / 8 launch rehearsed on ONE GPU (MPA_BENCH_ONE_GPU=1: every rank on GPU 0, so all
# ranks share one HBM and N = 1 is the ceiling): bench.py --gpus N self-launched, c2 (the default line) and c5.
set -u
R=$PWD
T=${1:-r06reh}
O=$R/gpurun_out/$T
mkdir -p $O
export MPA_BENCH_ONE_GPU=1
for c in c2 c5; do
  for n in 2 4 8; do
    if [ $c = c2 ]; then a="--steps 100 --warmup 10"; else a="--steps 10 --warmup 3"; fi
    timeout -k 10 400 python -u bench.py --gpus $n --config $c --no-cpu-baseline $a > $O/reh_${c}_n$n.log 2>&1 || { echo "$c N=$n failed"; tail -5 $O/reh_${c}_n$n.log; exit 1; }
    grep '^{' $O/reh_${c}_n$n.log | python3 -c "import json,sys;d=json.load(sys.stdin);r=d['roofline'];print('$c N=$n', d['value'], d['ms_per_step'], 'kernel', r.get('avg_launch_ms'), 'exchange', (d.get('exchange') or {}).get('avg_us'), 'path', d.get('payload_path'))"
  done
done
