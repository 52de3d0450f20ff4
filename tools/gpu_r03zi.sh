# Round 3, session 2: the launch round trip by kernel-argument size and a resident-kernel
# ping-pong (tools/launch_cost.hip), then the fused-head GPU test.
set -u
O=gpurun_out/r03zi
mkdir -p $O
timeout -k 10 60 tools/bin/launch_cost > $O/launch_cost.txt 2>&1 || { cat $O/launch_cost.txt; exit 1; }
cat $O/launch_cost.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "fused_head or timing" > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -2; exit $rc
