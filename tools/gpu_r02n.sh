# Round 2: where the one-GPU N=8 rehearsal spends its epoch (kernel trace of all 8 ranks)
set -u
R=$PWD
O=$R/gpurun_out/r02n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
MPA_BENCH_ONE_GPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/n8 -o n8 -- python3 $R/bench.py --gpus 8 --steps 30 --warmup 5 --no-cpu-baseline > $O/n8.log 2>&1 || exit $?
grep '^{' $O/n8.log | cut -c1-300
ls $O/n8 | head
