#!/bin/bash
# Round 6: armed two tasks deep (MPA_ARM_DEPTH=2, the default on a GPU rank 0 does not use).  The multi-process GPU
# tests (depth 1 and 2), then bench A/Bs of depth 1 / 2 / host-launched on one GPU: the node's per-GPU placement in
# miniature (c2n4 --gpus 2, 8192-row shards) and at the N = 4 shard size, and round 5's 7 + 1 placement.
set -u
R=$PWD
T=${1:-r06dep}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
(timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_procs.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/procs.log 2>&1) \
  || { echo "procs failed"; tail -30 $O/procs.log; exit 1; }
tail -3 $O/procs.log
run() {  # tag, config, steps, env...
  local tag=$1 cfg=$2 steps=$3; shift 3
  (cd /tmp && env MPA_WAIT_TIMEOUT_S=60 MPA_BENCH_ONE_GPU=1 "$@" timeout -k 10 240 python3 $R/bench.py --gpus 2 --config $cfg \
    --no-cpu-baseline --steps $steps --warmup 200 > $O/$tag.log 2>&1) || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  grep '^{' $O/$tag.log > $O/$tag.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['roofline'].get('avg_launch_ms'))" $O/$tag.json $tag
}
for rep in 1 2; do
  run mini_d1_$rep c2n4 3000 MPA_BENCH_ROWS=16384 MPA_ARM_DEPTH=1
  run mini_d2_$rep c2n4 3000 MPA_BENCH_ROWS=16384 MPA_ARM_DEPTH=2
  run mini_host_$rep c2n4 3000 MPA_BENCH_ROWS=16384 MPA_ARM=0
  run full_d1_$rep c2n4 1000 MPA_ARM_DEPTH=1
  run full_d2_$rep c2n4 1000 MPA_ARM_DEPTH=2
  run full_host_$rep c2n4 1000 MPA_ARM=0
  run p71_d1_$rep c2 3000 MPA_BENCH_ROWS=65536 MPA_BENCH_PLACEMENT=0,0,0,0,0,0,0,1 MPA_ARM_DEPTH=1
  run p71_d2_$rep c2 3000 MPA_BENCH_ROWS=65536 MPA_BENCH_PLACEMENT=0,0,0,0,0,0,0,1 MPA_ARM_DEPTH=2
done
echo "all ok"
