#!/bin/bash
# Round 6, follow-up 3: host event stamps (measurement build, MPA_HOST_STAMP) beside the kernel traces of the
# one-worker-per-rank miniature (c2n4 at --gpus 2 on one GPU, 8192-row shards), armed and host-launched
# (tools/arm_timeline.py).
set -u
R=$PWD
T=${1:-r06ctl4}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
ML=$R/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
trace() {  # tag, env...
  local tag=$1; shift
  mkdir -p $O/stamps_$tag
  (cd /tmp && env MPA_WAIT_TIMEOUT_S=60 MPA_BENCH_ONE_GPU=1 MPA_BENCH_ROWS=16384 MPA_LIB=$ML MPA_HOST_STAMP=$O/stamps_$tag "$@" \
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$tag -o %pid% -- \
    python3 $R/bench.py --gpus 2 --config c2n4 --no-cpu-baseline --steps 2000 --warmup 100 --timing-period 8 > $O/trace_$tag.log 2>&1) \
    || { echo "trace $tag failed"; tail -5 $O/trace_$tag.log; exit 1; }
  grep '^{' $O/trace_$tag.log > $O/trace_$tag.json
  python3 tools/arm_timeline.py $O/stamps_$tag $O/trace_$tag $O/trace_$tag.json --last 70 > $O/timeline_$tag.txt 2>&1 \
    || { echo "timeline $tag failed"; cat $O/timeline_$tag.txt; exit 1; }
  echo "== $tag $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" $O/trace_$tag.json)"
  tail -32 $O/timeline_$tag.txt
}
trace arm
trace host MPA_ARM=0
echo "all ok"
