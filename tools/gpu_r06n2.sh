#!/bin/bash
# Round 6: the two-process control-path budget (tools/n2_budget.py) with the remote completion
# word polled in rank 0's GPU memory (default) and in host memory (MPA_DONE_DEV=0), alternating on one box;
# c2 rehearsal shards, the node's per-remote-worker placement (rank 0 seven workers, rank 1 one, armed).
set -u
R=$PWD
T=${1:-r06n2}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for dd in 1 0; do
    tag=dd${dd}_$rep
    (cd /tmp && env MPA_DONE_DEV=$dd MPA_WAIT_TIMEOUT_S=60 MPA_BENCH_ONE_GPU=1 MPA_BENCH_ROWS=65536 MPA_BENCH_PLACEMENT=0,0,0,0,0,0,0,1 \
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$tag -o %pid% -- python3 $R/bench.py --gpus 2 --config c2 \
      --no-cpu-baseline --steps 2000 --warmup 100 > $O/trace_$tag.log 2>&1) || { echo "trace $tag failed"; tail -5 $O/trace_$tag.log; exit 1; }
    grep '^{' $O/trace_$tag.log > $O/trace_$tag.json
    python3 tools/n2_budget.py $O/trace_$tag $O/trace_$tag.json --epochs 1500 > $O/budget_$tag.txt 2>&1 || { echo "budget $tag failed"; cat $O/budget_$tag.txt; exit 1; }
    echo "$tag $(cat $O/budget_$tag.txt | tail -1)"
  done
done
