# Round 3, call 12: c5 same-box A/B of the LDS-DMA asm: s_nop 0 after the m0 write (nop), that
# plus m0 saved and restored around each DMA (full), neither (noasm), and 1a3da88
set -u
O=gpurun_out/r03l
mkdir -p $O
L=$PWD/mpistragglers.jl_amd
b() {  # label lib
  MPA_LIB=$2 timeout -k 10 240 python -u bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/$1.log 2>&1 || exit $?
  grep '^{' $O/$1.log > $O/$1.json
  echo "$1 $(python3 -c "import json;d=json.load(open('$O/$1.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])")"
}
for k in 1 2; do
  b nop$k $L/_build/libmpiasyncpools.so
  b full$k $L/_build_ab/lib_full.so
  b noasm$k $L/_build_ab/lib_noasm.so
  b old$k $L/_build_ab/lib_1a3da88.so
done
