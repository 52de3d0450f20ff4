# Round-end refresh of every committed number from ONE box: GPU tests, the N=1 bench (c2)
# and c1/c3/c4/c5 lines, then the c2 kernel trace + HBM counters (tools/gpu_profile.sh).
set -u
T=${TAG:-x}
CONFIGS="c1 c3 c4 c5" TAG=$T bash tools/gpu_full.sh || exit $?
TAG=$T bash tools/gpu_profile.sh || exit $?
