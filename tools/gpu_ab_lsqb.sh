# A/B of two builds of the library in ONE call (boxes differ by several %): the probe's
# per-pass kernel times with MPA_LIB=<other build> and with the in-tree build, alternating
set -u
R=$PWD
O=$R/gpurun_out/ab_${TAG:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  MPA_LIB=$R/mpistragglers.jl_amd/_build/ab/lib_before.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/before$k -o m -- python3 $R/tools/lsqb_mall_probe.py 262144 > $O/before$k.log 2>&1 || exit $?
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/after$k -o m -- python3 $R/tools/lsqb_mall_probe.py 262144 > $O/after$k.log 2>&1 || exit $?
done
cd $R && for k in 1 2; do echo "before $k"; python3 tools/pass_times.py $O/before$k 262144; echo "after $k"; python3 tools/pass_times.py $O/after$k 262144; done
