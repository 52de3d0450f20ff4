# lsqp7's L2-prefetch distance sweep against lsqp4, one box (measurement build)
set -u
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
bash tools/gpu.sh r05n var:p4:c5:--steps+20+--warmup+3 var:p7pf1:c5:MPA_LSQP7=1,MPA_LSQP_PF=1:--steps+20+--warmup+3 var:p7pf2:c5:MPA_LSQP7=1,MPA_LSQP_PF=2:--steps+20+--warmup+3 var:p7pf3:c5:MPA_LSQP7=1,MPA_LSQP_PF=3:--steps+20+--warmup+3 var:p7pf4:c5:MPA_LSQP7=1,MPA_LSQP_PF=4:--steps+20+--warmup+3 var:p4b:c5:--steps+20+--warmup+3
