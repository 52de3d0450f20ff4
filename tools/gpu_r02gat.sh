# Round 2 session 3: a server gathers a flush's doorbells (~2 us) into one launch vs MPA_GATHER=0

# (the multi-process GPU tests, then c2 at N = 2 / 4 on one GPU, same box)
set -u
O=gpurun_out/r02gat
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 180 --timeout-method thread > $O/dist.log 2>&1; rc=$?
grep -E "passed|failed" $O/dist.log | tail -1; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/dist.log | head; exit $rc; }
for r in 1 2; do for n in 2 4; do for v in 0 1; do
MPA_GATHER=$v MPA_BENCH_ONE_GPU=1 timeout -k 10 300 python3 -u bench.py --gpus $n --config c2 --steps 100 --warmup 10 --no-cpu-baseline > $O/n${n}_v$v.$r.log 2>&1 || exit $?
grep '^{' $O/n${n}_v$v.$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$n MPA_GATHER=$v', d['value'], d['ms_per_step'])"
done; done; done
