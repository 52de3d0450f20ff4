# Pass-1 ceiling probes (LSQB_P1_PROBE builds under _build/ab/): the in-tree build, then
# 1 = loads only, 2 = loads + MFMAs; per-pass medians at 8 workers x 262144 rows, one box.
set -u
R=$PWD
O=$R/gpurun_out/p1_${TAG:-x}
mkdir -p $O
if [ -n "${TESTS_ENV:-}" ]; then
  env $TESTS_ENV timeout -k 10 300 python -u -m pytest tests/test_gpu_lsqb.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  echo "lsqb tests ($TESTS_ENV) rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  for v in ${VARIANTS:-base p1probe1 p1probe2}; do
    P1=
    if [ $v = base ] || [ $v = async ] || [ $v = pair ]; then L=$R/mpistragglers.jl_amd/_build/libmpiasyncpools.so; else L=$R/mpistragglers.jl_amd/_build/ab/$v/libmpiasyncpools.so; fi
    { [ $v = async ] || [ $v = pair ]; } && P1=$v
    MPA_LSQB_P1=$P1 MPA_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$v$k -o m -- python3 $R/tools/lsqb_mall_probe.py 262144 > $O/$v$k.log 2>&1 || exit $?
  done
done
cd $R && for k in 1 2; do for v in ${VARIANTS:-base p1probe1 p1probe2}; do echo "$v $k: $(python3 tools/pass_times.py $O/$v$k 262144)"; done; done
