# c2 with 32 KiB per wave and tile (rb8, MPA_LSQ_VARIANT=14) and 24 KiB (rb6, 15) against the shipped rb4 (0), alternating
# (measurement build); then the product's batched 2048-column path: its parity tests and the c3k line
set -u
TESTS_TAG=_2048 bash tools/gpu.sh r05ac tests:batched_2048+or+test_lsq_f32 bench:c3k:--steps+20+--warmup+3+--no-cpu-baseline || exit $?
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
bash tools/gpu.sh r05ac var:v0a:c2:MPA_LSQ_VARIANT=0 var:v14a:c2:MPA_LSQ_VARIANT=14 var:v15a:c2:MPA_LSQ_VARIANT=15 \
  var:v0b:c2:MPA_LSQ_VARIANT=0 var:v14b:c2:MPA_LSQ_VARIANT=14 var:v15b:c2:MPA_LSQ_VARIANT=15 \
  var:v14g256:c2:MPA_LSQ_VARIANT=14,MPA_LSQ_GRID=256 var:v14g128:c2:MPA_LSQ_VARIANT=14,MPA_LSQ_GRID=128 var:v0c:c2:MPA_LSQ_VARIANT=0
