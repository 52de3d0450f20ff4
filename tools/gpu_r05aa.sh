# the 2048-column lsq_grad_kernel variants (measurement build, MPA_LSQ_V2048): c4k / c3k (one batched launch per epoch)
set -u
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
A=--steps+20+--warmup+3
bash tools/gpu.sh r05aa var:c4k_v0:c4k:MPA_LSQ_V2048=0:$A var:c4k_v1:c4k:MPA_LSQ_V2048=1:$A var:c4k_v2:c4k:MPA_LSQ_V2048=2:$A var:c4k_v3:c4k:MPA_LSQ_V2048=3:$A var:c4k_v4:c4k:MPA_LSQ_V2048=4:$A var:c4k_v0b:c4k:MPA_LSQ_V2048=0:$A \
  var:c3k_v0:c3k:MPA_LSQ_V2048=0:$A var:c3k_v1:c3k:MPA_LSQ_V2048=1:$A var:c3k_v2:c3k:MPA_LSQ_V2048=2:$A var:c3k_v3:c3k:MPA_LSQ_V2048=3:$A var:c3k_v4:c3k:MPA_LSQ_V2048=4:$A var:c3k_v5:c3k:MPA_LSQ_V2048=5:$A var:c3k_v0b:c3k:MPA_LSQ_V2048=0:$A \
  var:c4_v0:c4:MPA_LSQ_V2048=0 var:c4_v1:c4:MPA_LSQ_V2048=1 var:c4_v3:c4:MPA_LSQ_V2048=3 var:c3_v0:c3:MPA_LSQ_V2048=0 var:c3_v3:c3:MPA_LSQ_V2048=3
