# lsqp7 (measurement build) parity, then a same-box A/B against lsqp4
set -u
export MPA_LIB=$PWD/mpistragglers.jl_amd/_build_measure/libmpiasyncpools.so
mkdir -p gpurun_out/r05m
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsqb.py -m gpu -v -x --timeout 240 --timeout-method thread -k "pair_step or lsqp4_pairs_default or full_form" > gpurun_out/r05m/tests.log 2>&1 || { tail -30 gpurun_out/r05m/tests.log; exit 1; }
tail -3 gpurun_out/r05m/tests.log
bash tools/gpu.sh r05m abenv:c5:3:MPA_LSQP7=1:--steps+20+--warmup+3
