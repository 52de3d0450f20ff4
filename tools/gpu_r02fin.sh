# Round 2 session 3: host-launched remote tasks by default (pre-arming opt-in): the full GPU
# suite (armed paths via MPA_ARM), then one-GPU rehearsals of the scaling path (N = 2, 4)
set -u
O=gpurun_out/r02fin
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
grep -E "^(FAILED)|passed|failed" $O/gpu_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
for n in 2 4; do for c in c2 c1; do
MPA_BENCH_ONE_GPU=1 timeout -k 10 300 python3 -u bench.py --gpus $n --config $c --steps 100 --warmup 10 --no-cpu-baseline > $O/n${n}_$c.log 2>&1 || exit $?
grep '^{' $O/n${n}_$c.log > $O/n${n}_$c.json; python3 -c "import json; d=json.load(open('$O/n${n}_$c.json')); print('$c N=$n', d['value'], d['ms_per_step'], d['exchange']['avg_us'])"
done; done
