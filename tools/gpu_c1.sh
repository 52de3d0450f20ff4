# c1 (k-of-n, latency-bound) bench and kernel timeline; MPA_COORD_BATCH A/B
set -u
R=$PWD
O=$R/gpurun_out/c1_${TAG:-x}
mkdir -p $O
for cb in 1 0; do
  MPA_COORD_BATCH=$cb timeout -k 10 200 python -u bench.py --config c1 --no-cpu-baseline > $O/bench_cb$cb.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o c1 -- python3 $R/bench.py --config c1 --steps 200 --warmup 20 --no-cpu-baseline > $O/trace.log 2>&1 || exit $?
cd $R && for cb in 1 0; do tail -1 $O/bench_cb$cb.log | cut -c1-220; done
