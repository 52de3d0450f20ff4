# the epoch step's chunk loads no longer wait for the iterate's load (a hidden pad address for
# chunks past n): the whole -m gpu suite, same-box A/Bs against the library before this round's
# head changes (_build_ab), c5's line, then the device-side head split (measurement build)
set -u
KEEP_GOING=1 bash tools/gpu.sh r05bd smoke tests || exit $?
bash tools/gpu.sh r05bd ab:c1:3:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so ab:c2:2:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so bench:c5 || exit $?
MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so MPA_HEAD_STAMP=1 bash tools/gpu.sh r05bd py:c1_trace.py:3000
