# the fused-head variant's b values loaded with its tile (before the token wait): the whole -m gpu
# suite, same-box A/Bs against the library before this round's head changes (_build_ab), then the
# device-side head split (measurement build)
set -u
KEEP_GOING=1 bash tools/gpu.sh r05bf smoke tests || exit $?
bash tools/gpu.sh r05bf ab:c1:3:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so ab:c2:1:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so || exit $?
MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so MPA_HEAD_STAMP=1 bash tools/gpu.sh r05bf py:c1_trace.py:3000
