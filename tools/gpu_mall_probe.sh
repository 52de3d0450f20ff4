# Infinity-Cache probe for a row-chunked c5 schedule: GPU tests + c2 bench first (tree
# health), then probe_c5_mall.py at several rows/worker under rocprofv3 kernel stats.
set -u
R=$PWD
T=${TAG:-x}
O=$R/gpurun_out/mall_$T
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py > $O/bench_c2.log 2>&1; rc=$?
echo "bench c2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp
for rows in ${ROWS:-4096 8192 16384 131072}; do
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$rows -o p -- python3 $R/tools/probe_c5_mall.py $rows 40 > $O/probe_$rows.log 2>&1; rc=$?
echo "probe $rows rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
