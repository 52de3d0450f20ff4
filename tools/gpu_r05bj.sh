# the one-level tree's last reducer issues its partial loads at once (clamped) and reads the cancel
# word while they are in flight: the whole -m gpu suite, same-box A/Bs against _build_ab, then the
# device-side head split (measurement build)
set -u
KEEP_GOING=1 bash tools/gpu.sh r05bj smoke tests || exit $?
bash tools/gpu.sh r05bj ab:c1:3:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so ab:c2:2:$PWD/mpistragglers.jl_amd/_build_ab/libmpiasyncpools.so || exit $?
MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so MPA_HEAD_STAMP=1 bash tools/gpu.sh r05bj py:c1_trace.py:3000
