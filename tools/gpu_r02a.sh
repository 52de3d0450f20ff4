# Round 2, first GPU pass: the whole GPU suite (incl. the new c1/c4 oracle tests), the N=1
# bench line, then the multi-process path rehearsed on one GPU: `bench.py --gpus 2`
# self-launched, and N = 8 with lazily created streams vs the round-1 eager streams.
set -u
O=gpurun_out/r02a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py > $O/bench_c2.log 2>&1; rc=$?
echo "bench c2 rc=$rc"; tail -1 $O/bench_c2.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
# fused tail A/B on the same box (default = tail on), B A B A
for t in 0 1 0 1; do
MPA_TAIL=$t timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 300 --warmup 30 > $O/bench_tail$t.log 2>&1; rc=$?
echo "tail=$t rc=$rc $(python3 -c "import json,sys;d=json.loads(open('$O/bench_tail$t.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['exchange'])")"; [ $rc -eq 0 ] || exit $rc
done
MPA_BENCH_ONE_GPU=1 MPA_WAIT_TIMEOUT_S=60 timeout -k 10 300 python -u bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline > $O/n2_self.log 2>&1; rc=$?
echo "n2 self-launch rc=$rc"; grep -c '^{' $O/n2_self.log; tail -1 $O/n2_self.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
for mode in lazy eager; do
E=0; [ $mode = eager ] && E=1
MPA_EAGER_STREAMS=$E MPA_BENCH_ONE_GPU=1 MPA_WAIT_TIMEOUT_S=60 timeout -k 10 300 python -u bench.py --gpus 8 --steps 50 --warmup 5 > $O/n8_$mode.log 2>&1; rc=$?
echo "n8 $mode rc=$rc"; tail -1 $O/n8_$mode.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
