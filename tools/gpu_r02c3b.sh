# Round 2 session 3: N=1 lines of c1, c3, c4 on the final tree (after the out-of-row clamp fix)
# on GPU 0) for c2 and c5; whether this image's MPICH is present on the box
set -u
O=gpurun_out/r02c3b
mkdir -p $O
ls -la /opt/conda/bin/mpiexec /opt/conda/include/mpi.h > $O/mpich.txt 2>&1; echo "mpich: $(head -2 $O/mpich.txt | tr '\n' ' ')"
for c in c1 c3 c4; do
timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 > $O/bench_$c.log 2>&1; rc=$?
echo "bench $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{' $O/bench_$c.log > $O/bench_$c.json; cut -c1-160 $O/bench_$c.json
done
