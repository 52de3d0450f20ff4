# c1's pre-armed head with its own arguments staged in LDS before the go wait: the head / pre-armed
# tests, a same-box A/B against the previous library (_build_ab), the device-side head split
set -u
bash tools/gpu.sh r05ax tests:head+or+prearm+or+kmap2+or+fused+or+native ab:c1:3:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so ab:c2:1:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so || exit $?
MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so MPA_HEAD_STAMP=1 bash tools/gpu.sh r05ax py:c1_trace.py:3000
