# the round-5 tree: smoke, the whole -m gpu suite, every bench line; then c1's fused-head launch stamped on the
# device (measurement build, MPA_HEAD_STAMP=1)
set -u
KEEP_GOING=1 bash tools/gpu.sh r05ap smoke tests bench:c2 bench:c1 bench:c3 bench:c4 bench:c5
MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so MPA_HEAD_STAMP=1 bash tools/gpu.sh r05ap py:c1_trace.py:3000
