# Round 3, session 2: the N-process bench path rehearsed on one GPU (every rank on GPU 0, shared
# HBM and CUs: N = 1 is the ceiling) with the round-3 defaults (device-armed tasks where a process
# serves one worker: N = 8; cross-process fused tail) against MPA_ARM=0; c2 and c1
# (profiles/r03_rehearsal_n248.txt)
set -u
O=gpurun_out/r03z
mkdir -p $O
run() {  # label n config env...
  local lab=$1 n=$2 c=$3; shift 3
  env "$@" MPA_BENCH_ONE_GPU=1 MPA_WAIT_TIMEOUT_S=60 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus $n --config $c --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline > $O/$lab.log 2>&1; rc=$?
  echo "$lab rc=$rc $(grep '^{' $O/$lab.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
}
for k in 1 2; do
  run n2_c2_$k 2 c2 MPA_X=1
  run n4_c2_$k 4 c2 MPA_X=1
  run n8_c2_$k 8 c2 MPA_X=1
  run n8_c2_arm0_$k 8 c2 MPA_ARM=0
  run n8_c1_$k 8 c1 MPA_X=1
done
