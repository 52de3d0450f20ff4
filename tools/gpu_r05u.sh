# c3k / c4k (c3's and c4's task shapes, nwait = n, no delays): the batched launch's grid (measurement build)
set -u
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
A=--steps+20+--warmup+3
bash tools/gpu.sh r05u var:c3k192:c3k:MPA_LSQ_GRID=192:$A var:c3k384:c3k:MPA_LSQ_GRID=384:$A var:c3k512:c3k:MPA_LSQ_GRID=512:$A var:c3k768:c3k:MPA_LSQ_GRID=768:$A var:c3k1024:c3k:MPA_LSQ_GRID=1024:$A \
  var:c4k192:c4k:MPA_LSQ_GRID=192:$A var:c4k384:c4k:MPA_LSQ_GRID=384:$A var:c4k512:c4k:MPA_LSQ_GRID=512:$A var:c4k768:c4k:MPA_LSQ_GRID=768:$A var:c4k1024:c4k:MPA_LSQ_GRID=1024:$A \
  var:c2g192:c2:MPA_LSQ_GRID=192:$A var:c2g384:c2:MPA_LSQ_GRID=384:$A
