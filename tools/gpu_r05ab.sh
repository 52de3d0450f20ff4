# fp32 2048 columns: RB = 4 (MPA_LSQ_V2048=2) against the shipped RB = 2, alternating on one box (measurement build)
set -u
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
A=--steps+20+--warmup+3
bash tools/gpu.sh r05ab abenv:c3:3:MPA_LSQ_V2048=2 abenv:c3k:2:MPA_LSQ_V2048=2:$A
