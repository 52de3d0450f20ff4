# the fp64 fused-head variant only loads b with its tile (fp32 back to per-row loads, bitwise with
# the plain variant): the whole -m gpu suite, same-box A/Bs against the library before this
# round's head changes (_build_ab), then the device-side head split (measurement build)
set -u
KEEP_GOING=1 bash tools/gpu.sh r05bg smoke tests || exit $?
bash tools/gpu.sh r05bg ab:c1:3:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so ab:c2:2:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so || exit $?
MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so MPA_HEAD_STAMP=1 bash tools/gpu.sh r05bg py:c1_trace.py:3000
