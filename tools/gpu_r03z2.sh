# Round 3, session 2: the N = 8 one-GPU rehearsal regression (c2: 788 it/s in round 2, 64 now):
# the round-3 tree with MPA_TAIL=0 and/or MPA_ARM=0 against the round-2 final tree (b72e083,
# _bisect/r02); bounded waits of 30 s (profiles/r03_rehearsal_n248.txt)
set -u
R=$PWD
O=$R/gpurun_out/r03z2
mkdir -p $O
run() {  # label dir env...
  local lab=$1 dir=$2; shift 2
  (cd $dir && env "$@" MPA_BENCH_ONE_GPU=1 MPA_WAIT_TIMEOUT_S=30 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 8 --config c2 --steps 50 --warmup 5 --no-cpu-baseline) > $O/$lab.log 2>&1; rc=$?
  echo "$lab rc=$rc $(grep '^{' $O/$lab.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])" 2>/dev/null)"
}
run r02 $R/_bisect/r02 MPA_X=1
run tail0_arm0 $R MPA_TAIL=0 MPA_ARM=0
run arm0 $R MPA_ARM=0
run tail0 $R MPA_TAIL=0
run default $R MPA_X=1
