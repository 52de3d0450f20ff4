# Round 2 session 3: the go word read by the reply's writer only (pre-armed tasks no longer
# read host memory before they start): multi-process GPU tests (armed paths and cancels),
# then armed vs host-launched c1 / c2 at N = 2 on one GPU, twice, same box
set -u
O=gpurun_out/r02arm2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_capi_client.py -x -v --timeout 180 --timeout-method thread > $O/dist.log 2>&1; rc=$?
grep -E "passed|failed" $O/dist.log | tail -1; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/dist.log | head; exit $rc; }
for r in 1 2; do for c in c1 c2; do for arm in 0 1; do
MPA_ARM=$arm MPA_BENCH_ONE_GPU=1 timeout -k 10 300 python3 -u bench.py --gpus 2 --config $c --steps 100 --warmup 10 --no-cpu-baseline > $O/${c}_arm$arm.$r.log 2>&1 || exit $?
grep '^{' $O/${c}_arm$arm.$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c N=2 MPA_ARM=$arm run $r', d['value'], d['ms_per_step'])"
done; done; done
