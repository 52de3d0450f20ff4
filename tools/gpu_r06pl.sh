#!/bin/bash
# Round 6: the N = 7 one-GPU line (placement 0,0,1,2,3,4,5,6: rank 0 two workers, six armed one-worker ranks) stops in
# its timed session: rank 0 waits past MPA_WAIT_TIMEOUT_S for a worker (r06pl).  Small shards, 300 timed epochs after a
# pause, with: the library before round 6's two-deep arming (_build_old, tree b1cef4d), host-launched servers
# (MPA_ARM=0), no fused tail (MPA_TAIL=0), and the current library again.  A step that ends with the transport's own
# timeout error (rc 1) lets the next one run; a time limit ends the call.
set -u
O=gpurun_out/${1:-r06pl2}; mkdir -p $O
export MPA_BENCH_ONE_GPU=1 MPA_BENCH_ROWS=65536 MPA_WAIT_TIMEOUT_S=20
run() {  # tag, env...
  local tag=$1; shift
  env "$@" MPA_BENCH_PLACEMENT=0,0,1,2,3,4,5,6 timeout -k 10 100 python -u bench.py --gpus 7 --config c2 --no-cpu-baseline --steps 300 --warmup 20 > $O/$tag.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "$tag rc=$rc: $(grep -o 'DeviceError.*' $O/$tag.log | head -1)"
    if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
    return 0
  fi
  grep '^{' $O/$tag.log | python3 -c "import json,sys;d=json.load(sys.stdin);print('$tag', d['value'], d['ms_per_step'])"
}
run old MPA_LIB=$PWD/mpistragglers.jl_amd/_build_old/libmpiasyncpools.so
run host MPA_ARM=0
run notail MPA_TAIL=0
run cur MPA_X=0
echo "all ok"
