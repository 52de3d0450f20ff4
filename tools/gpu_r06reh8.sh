#!/bin/bash
# Round 6: the one-GPU N = 8 rehearsal (8 processes on GPU 0), device-armed (default) against host-launched (MPA_ARM=0).
set -u
O=gpurun_out/r06reh8; mkdir -p $O
export MPA_BENCH_ONE_GPU=1
for rep in 1 2; do
for c in c2 c5; do
  for arm in 2 0; do
    if [ $c = c2 ]; then a="--steps 100 --warmup 10"; else a="--steps 10 --warmup 3"; fi
    MPA_ARM=$arm timeout -k 10 300 python -u bench.py --gpus 8 --config $c --no-cpu-baseline $a > $O/${c}_arm${arm}_$rep.log 2>&1 || { echo "$c arm $arm failed"; tail -5 $O/${c}_arm${arm}_$rep.log; exit 1; }
    grep '^{' $O/${c}_arm${arm}_$rep.log | python3 -c "import json,sys;d=json.load(sys.stdin);r=d['roofline'];print('$c N=8 MPA_ARM=$arm', d['value'], d['ms_per_step'], 'kernel', r.get('avg_launch_ms'), 'exchange', (d.get('exchange') or {}).get('avg_us'))"
  done
done
done
