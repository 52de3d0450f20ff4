#!/bin/bash
# Round 6, follow-up 2 (tools/gpu_r06ctl.sh, gpu_r06ctl2.sh): the device-armed path against the host-launched one
# (MPA_ARM=0) in the node's per-GPU placement (one worker per rank: c2n4 at --gpus 2 on one GPU), with the bench's
# usual HIP-event sampling (one launch in 8) instead of every launch, in miniature (8192-row shards) and at the
# node's N = 4 shard size (2^17 rows, 512 MiB per task; both ranks share the one GPU's HBM here).
set -u
R=$PWD
T=${1:-r06ctl3}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
ML=$R/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
run() {  # tag, steps, env...
  local tag=$1 steps=$2; shift 2
  (cd /tmp && env MPA_WAIT_TIMEOUT_S=60 MPA_BENCH_ONE_GPU=1 "$@" timeout -k 10 240 python3 $R/bench.py --gpus 2 --config c2n4 \
    --no-cpu-baseline --steps $steps --warmup 200 --timing-period 8 > $O/$tag.log 2>&1) || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  grep '^{' $O/$tag.log > $O/$tag.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['roofline'].get('avg_launch_ms'), (d.get('exchange') or {}).get('avg_us'))" $O/$tag.json $tag
}
for rep in 1 2; do
  run mini_arm_$rep 3000 MPA_BENCH_ROWS=16384
  run mini_host_$rep 3000 MPA_BENCH_ROWS=16384 MPA_ARM=0
  run full_arm_$rep 1000
  run full_host_$rep 1000 MPA_ARM=0
  run full_kern_$rep 1000 MPA_LIB=$ML MPA_ARM_WAIT=kernel MPA_ARM_WAIT_FORCE=1
done
echo "all ok"
