# same-box A/B of the c5 bench: pass-1 grid 256 vs the default (512), alternating
set -u
O=gpurun_out/c5ab_${TAG:-x}
mkdir -p $O
for k in 1 2; do for g in 256 512; do
  MPA_LSQB_GRID1=$g timeout -k 10 200 python -u bench.py --config c5 --steps 30 --warmup 3 > $O/g${g}_$k.log 2>&1 || exit $?
  echo "grid1=$g run $k: $(grep '^{' $O/g${g}_$k.log | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], 'it/s', d['roofline']['avg_launch_ms'], 'ms/launch')")"
done; done
