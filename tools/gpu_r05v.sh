# c3 (delayed single-task launches) under the batched-launch grid candidates (measurement build)
set -u
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
bash tools/gpu.sh r05v var:c3g192a:c3:MPA_LSQ_GRID=192 var:c3g384a:c3:MPA_LSQ_GRID=384 var:c3g512a:c3:MPA_LSQ_GRID=512 \
  var:c3g192b:c3:MPA_LSQ_GRID=192 var:c3g384b:c3:MPA_LSQ_GRID=384 var:c3g512b:c3:MPA_LSQ_GRID=512 \
  var:c4g192:c4:MPA_LSQ_GRID=192 var:c4g384:c4:MPA_LSQ_GRID=384 var:c3kg512:c3k:MPA_LSQ_GRID=512:--steps+20+--warmup+3 var:c2g192:c2:MPA_LSQ_GRID=192
