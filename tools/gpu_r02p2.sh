# Round 2: SQ counters of the strip-ring lsqp4 (isolated 8-task launches): where its waves wait
set -u
R=$PWD
O=$R/gpurun_out/r02p2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS --output-format csv -d $O/p1 -o p -- python3 $R/tools/lsqb_mall_probe.py 1048576 > $O/p1.log 2>&1 || exit $?
echo pass1 ok
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d $O/p2 -o p -- python3 $R/tools/lsqb_mall_probe.py 1048576 > $O/p2.log 2>&1 || exit $?
echo pass2 ok
