# Round 2 session 3: kernel timeline of the cross-process path (both ranks on GPU 0): c1 at N=2
set -u
R=$PWD
O=$R/gpurun_out/r02tl_c2b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
MPA_BENCH_ONE_GPU=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o tr_%pid% -- python3 $R/bench.py --gpus 2 --config c2 --steps 40 --warmup 5 --no-cpu-baseline > $O/run.log 2>&1 || exit $?
ls -R $O/tr | head -20
