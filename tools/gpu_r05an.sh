# c1's coordinator thread, profiled on the host (measurement build, MPA_HOST_PROF=1)
set -u
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so MPA_HOST_PROF=1
bash tools/gpu.sh r05an py:c1_trace.py:3000
