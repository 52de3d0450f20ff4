# remote messages written through at system scope (EpochArgs::dst_sys) against round 4's per-block system-scope
# release (MPA_MSG_WT=0): the multi-process parity tests, then N = 2 on one GPU with rehearsal shards (c5, c2)
set -u
TESTS_TAG=_procs bash tools/gpu.sh r05y tests:test_gpu_procs || exit $?
export MPA_BENCH_ONE_GPU=1 MPA_BENCH_ROWS=65536
bash tools/gpu.sh r05y abenv:c5:3:MPA_MSG_WT=0:--gpus+2+--steps+200+--warmup+20 abenv:c2:2:MPA_MSG_WT=0:--gpus+2+--steps+300+--warmup+30
