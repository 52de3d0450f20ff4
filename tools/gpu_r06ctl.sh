#!/bin/bash
# Round 6: the per-GPU control path of the node's placement in miniature.  bench.py --gpus 2
# --config c2n4 on ONE GPU with 8192-row shards (MPA_BENCH_ROWS=16384): rank 0 serves one worker (fused tail), rank 1
# one (device-armed), as every GPU of the 8-GPU node does, with tasks so small that the epoch is mostly control path.
# Alternating on one box: the product's armed wait (one-wave door_wait_kernel, the task queued behind it), the
# measurement build's same path, its in-kernel wait (MPA_ARM_WAIT=kernel, forced onto the shared GPU), and the
# host-launched task (MPA_ARM=0).  Then kernel traces of the door_wait and in-kernel forms (tools/n2_budget.py).
set -u
R=$PWD
T=${1:-r06ctl}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
ML=$R/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
common="MPA_WAIT_TIMEOUT_S=60 MPA_BENCH_ONE_GPU=1 MPA_BENCH_ROWS=16384"
run() {  # tag, env...
  local tag=$1; shift
  (cd /tmp && env $common "$@" timeout -k 10 180 python3 $R/bench.py --gpus 2 --config c2n4 --no-cpu-baseline \
    --steps 3000 --warmup 300 > $O/$tag.log 2>&1) || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  grep '^{' $O/$tag.log > $O/$tag.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], (d.get('exchange') or {}).get('avg_us'))" $O/$tag.json $tag
}
for rep in 1 2; do
  run prod_$rep
  run meas_$rep MPA_LIB=$ML
  run kern_$rep MPA_LIB=$ML MPA_ARM_WAIT=kernel MPA_ARM_WAIT_FORCE=1
  run host_$rep MPA_ARM=0
done
trace() {  # tag, env...
  local tag=$1; shift
  (cd /tmp && env $common "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$tag -o %pid% -- \
    python3 $R/bench.py --gpus 2 --config c2n4 --no-cpu-baseline --steps 2000 --warmup 100 > $O/trace_$tag.log 2>&1) \
    || { echo "trace $tag failed"; tail -5 $O/trace_$tag.log; exit 1; }
  grep '^{' $O/trace_$tag.log > $O/trace_$tag.json
  python3 tools/n2_budget.py $O/trace_$tag $O/trace_$tag.json --epochs 1500 > $O/budget_$tag.txt 2>&1 \
    || { echo "budget $tag failed"; cat $O/budget_$tag.txt; exit 1; }
  echo "$tag"; cat $O/budget_$tag.txt
}
trace wave MPA_LIB=$ML
trace kern MPA_LIB=$ML MPA_ARM_WAIT=kernel MPA_ARM_WAIT_FORCE=1
echo "all ok"
