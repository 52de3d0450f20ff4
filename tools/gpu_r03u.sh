# Round 3, session 2: SQ counters of lsqp4 v4 on the c5 bench (two rocprofv3 --pmc passes, each
# its own run; profiles/r03_c5_sq_counters.txt)
set -u
R=$PWD
O=$R/gpurun_out/r03u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/p1 -o c5 -- python3 $R/bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline > $O/p1.log 2>&1 || exit $?
echo p1 ok
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT --output-format csv -d $O/p2 -o c5 -- python3 $R/bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline > $O/p2.log 2>&1 || exit $?
echo p2 ok
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_EXP SQ_INSTS_BRANCH SQ_WAVES --output-format csv -d $O/p3 -o c5 -- python3 $R/bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline > $O/p3.log 2>&1 || echo "p3 failed (optional)"
ls $O/p1 $O/p2
