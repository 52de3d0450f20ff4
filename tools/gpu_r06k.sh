set -u
KEEP_GOING=1 bash tools/gpu.sh r06k tests:test_gpu_procs+or+past_cap+or+running_straggler || exit $?
export MPA_BENCH_ONE_GPU=1
bash tools/gpu.sh r06k bench:c5:--gpus+2+--steps+30+--warmup+5 abenv:c5:1:MPA_RESERVE_CUS=0:--gpus+2+--steps+30+--warmup+5 bench:c2:--gpus+2+--steps+200+--warmup+20
