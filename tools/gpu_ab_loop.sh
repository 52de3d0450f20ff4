# A/B of the native descent loop modes on the c2 bench, interleaved (one bench process each).
set -u
O=gpurun_out/ab_${TAG:-x}
mkdir -p $O
for k in 1 2; do
for m in ahead fuse noahead; do
case $m in ahead) E="";; noahead) E="MPA_AHEAD=0";; fuse) E="MPA_FUSE=0";; esac
env $E timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 400 > $O/${m}_$k.log 2>&1 || exit $?
echo "$m $k ok"
done
done
