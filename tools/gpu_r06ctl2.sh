#!/bin/bash
# Round 6, follow-up of tools/gpu_r06ctl.sh: in the node's per-GPU placement in miniature (c2n4 at --gpus 2 on one
# GPU, 8192-row shards) the device-armed path ran 0.134 ms per epoch against 0.038 host-launched.  Which part of the
# armed path costs it: bench lines of the armed path with the fused tail off (MPA_TAIL=0: rank 0 waits in
# wait_words_kernel + epoch_kernel), with the remote completion word in host memory (MPA_DONE_DEV=0), and of round
# 5's 7 + 1 placement (c2, 65536 rows) armed and host-launched; kernel traces of the host-launched and tail-off forms.
set -u
R=$PWD
T=${1:-r06ctl2}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
common="MPA_WAIT_TIMEOUT_S=60 MPA_BENCH_ONE_GPU=1"
run() {  # tag, config, rows, env...
  local tag=$1 cfg=$2 rows=$3; shift 3
  (cd /tmp && env $common MPA_BENCH_ROWS=$rows "$@" timeout -k 10 180 python3 $R/bench.py --gpus 2 --config $cfg \
    --no-cpu-baseline --steps 3000 --warmup 300 > $O/$tag.log 2>&1) || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  grep '^{' $O/$tag.log > $O/$tag.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], (d.get('exchange') or {}).get('avg_us'))" $O/$tag.json $tag
}
for rep in 1 2; do
  run arm_$rep c2n4 16384
  run host_$rep c2n4 16384 MPA_ARM=0
  run notail_$rep c2n4 16384 MPA_TAIL=0
  run ddhost_$rep c2n4 16384 MPA_DONE_DEV=0
  run p71arm_$rep c2 65536 MPA_BENCH_PLACEMENT=0,0,0,0,0,0,0,1
  run p71host_$rep c2 65536 MPA_BENCH_PLACEMENT=0,0,0,0,0,0,0,1 MPA_ARM=0
done
trace() {  # tag, env...
  local tag=$1; shift
  (cd /tmp && env $common MPA_BENCH_ROWS=16384 "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$tag -o %pid% -- \
    python3 $R/bench.py --gpus 2 --config c2n4 --no-cpu-baseline --steps 2000 --warmup 100 > $O/trace_$tag.log 2>&1) \
    || { echo "trace $tag failed"; tail -5 $O/trace_$tag.log; exit 1; }
  grep '^{' $O/trace_$tag.log > $O/trace_$tag.json
  echo "trace $tag ok"
}
trace host MPA_ARM=0
trace notail MPA_TAIL=0
echo "all ok"
