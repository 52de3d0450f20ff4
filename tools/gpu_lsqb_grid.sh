# c5 pass-1 / pass-2 launch-grid sweep in ONE call (MPA_LSQB_GRID1 / MPA_LSQB_GRID2), probe
# sizes 8 workers x 262144 rows x 2048 cols bf16; per-pass medians via tools/pass_times.py
set -u
R=$PWD
O=$R/gpurun_out/grid_${TAG:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-256:512 512:512 1024:512 256:1024 512:1024 256:512}; do
  g1=${cfg%%:*}; g2=${cfg##*:}; k=g${g1}_${g2}_$RANDOM
  MPA_LSQB_GRID1=$g1 MPA_LSQB_GRID2=$g2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$k -o m -- python3 $R/tools/lsqb_mall_probe.py 262144 > $O/$k.log 2>&1 || exit $?
  echo "grid1=$g1 grid2=$g2: $(cd $R && python3 tools/pass_times.py $O/$k 262144)"
done
