# Round 2 session 3: pre-armed remote tasks with the go word read once per wave, against
# host-launched remote tasks (MPA_ARM=0): c1 and c2 at N=2 with both ranks on GPU 0, traced
set -u
R=$PWD
O=$R/gpurun_out/r02arm
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for arm in 1 0; do
MPA_ARM=$arm MPA_BENCH_ONE_GPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_arm$arm -o tr_%pid% -- python3 $R/bench.py --gpus 2 --config c1 --steps 100 --warmup 10 --no-cpu-baseline > $O/c1_arm$arm.log 2>&1 || exit $?
echo "c1 arm=$arm $(grep '^{' $O/c1_arm$arm.log | cut -c100-200)"
done
cd $R
for arm in 1 0; do
MPA_ARM=$arm MPA_BENCH_ONE_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --config c2 --steps 50 --warmup 5 --no-cpu-baseline > $O/c2_arm$arm.log 2>&1 || exit $?
echo "c2 arm=$arm $(grep '^{' $O/c2_arm$arm.log | cut -c100-200)"
done
