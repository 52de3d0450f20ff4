# Round 2 session 3, final tree (after the go-word change): smoke, full GPU suite, c2 bench
set -u
O=${O:-gpurun_out/r02end2}
mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
grep -E "^(FAILED)|passed|failed" $O/gpu_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.log 2>&1 || exit $?
grep '^{' $O/bench_c2.log > $O/bench_n1.json; python3 -c "import json; d=json.load(open('$O/bench_n1.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'])"
