# the epoch step's loads and stores through the global address space (no flat ops: c1's pre-armed
# head read its LDS-staged arguments between serialised flat loads); the whole -m gpu suite, then
# same-box A/Bs against the library before this round's two head changes (_build_ab), then the
# device-side head split (measurement build)
set -u
KEEP_GOING=1 bash tools/gpu.sh r05az smoke tests || exit $?
bash tools/gpu.sh r05az ab:c1:3:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so ab:c2:2:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so || exit $?
MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so MPA_HEAD_STAMP=1 bash tools/gpu.sh r05az py:c1_trace.py:3000
