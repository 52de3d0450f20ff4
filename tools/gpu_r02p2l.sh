# Round 2 session 3: same-box A/B of the lsqp4 read-ahead knobs (phase-2 lookahead P2L 1 vs the
# shipped 2, phase-1 read-ahead AD 3/4/6), isolated 8-task c5 launches, alternating builds
# (profiles/r02_c5_strip_ring.txt)
set -u
R=$PWD
O=$R/gpurun_out/${OUT:-r02p2l}
mkdir -p $O
L=$R/mpistragglers.jl_amd
for r in 1 2 3; do for v in ${VARS:-default p1 ad3p1 ad6p1}; do
lib=$L/_build/libmpiasyncpools.so; [ $v != default ] && lib=$L/_build_ab/lib_$v.so
MPA_LIB=$lib timeout -k 10 200 python3 -u tools/lsqb_mall_probe.py 1048576 > $O/ab_$v$r.log 2>&1 || exit $?
echo "$v$r $(grep rows/ $O/ab_$v$r.log)"
done; done
