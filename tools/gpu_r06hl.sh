#!/bin/bash
# Round 6: where a server's host-launched task spends the serve thread's time (measurement build host stamps,
# tools/arm_timeline.py): doorbell seen (B) -> launch stream picked (p, q) -> hipLaunchKernel (k, K) -> T, in the
# one-worker-per-rank miniature (MPA_ARM=0) and in c2's default N = 2 placement (4 + 4 workers, one batch).
set -u
R=$PWD
T=${1:-r06hl}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
ML=$R/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
trace() {  # tag, config, rows, env...
  local tag=$1 cfg=$2 rows=$3; shift 3
  mkdir -p $O/stamps_$tag
  (cd /tmp && env MPA_WAIT_TIMEOUT_S=60 MPA_BENCH_ONE_GPU=1 MPA_BENCH_ROWS=$rows MPA_LIB=$ML MPA_HOST_STAMP=$O/stamps_$tag "$@" \
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$tag -o %pid% -- \
    python3 $R/bench.py --gpus 2 --config $cfg --no-cpu-baseline --steps 2000 --warmup 100 > $O/trace_$tag.log 2>&1) \
    || { echo "trace $tag failed"; tail -5 $O/trace_$tag.log; exit 1; }
  grep '^{' $O/trace_$tag.log > $O/trace_$tag.json
  python3 tools/arm_timeline.py $O/stamps_$tag $O/trace_$tag $O/trace_$tag.json --last 70 > $O/timeline_$tag.txt 2>&1 \
    || { echo "timeline $tag failed"; cat $O/timeline_$tag.txt; exit 1; }
  echo "== $tag $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" $O/trace_$tag.json)"
  tail -32 $O/timeline_$tag.txt
}
trace mini c2n4 16384 MPA_ARM=0
trace n2 c2 65536
echo "all ok"
