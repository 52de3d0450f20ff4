# Round 2 (session 2): the restored tree on a fresh box: smoke, full GPU suite, N=1 c2 bench line
set -u
R=$PWD
O=$R/gpurun_out/r02p
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
echo "$(tail -1 $O/smoke.log)"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "^(FAILED)|passed|failed" $O/gpu_tests.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench_c2.log 2>&1 || exit $?
grep '^{' $O/bench_c2.log > $O/bench_n1.json; echo "c2 $(cut -c1-300 $O/bench_n1.json)"
