# Round 2 session 3: lsqp4's strip DMAs with the nt policy bit vs default, same box, alternating
set -u
O=gpurun_out/r02nt
mkdir -p $O
L=$PWD/mpistragglers.jl_amd/_build_ab
for r in 1 2; do for v in base nt; do
MPA_LIB=$L/lib_$v.so timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/$v$r.log 2>&1 || exit $?
echo "$v $(grep rows/ $O/$v$r.log)"
done; done
