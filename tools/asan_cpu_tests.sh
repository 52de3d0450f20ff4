#!/bin/bash
# The CPU test suite against the library's host code built under AddressSanitizer and UBSan (make SAN=1 -> _build_asan;
# the GPU code is the usual build, and no test here launches it).  Run here, not on the GPU box.  The c1 MPI baseline
# test is left out: it asserts a rate, which the instrumented processes do not reach.
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
(cd "$R/mpistragglers.jl_amd" && make SAN=1 -j8 > /dev/null) || exit $?
cd "$R"
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 MPA_LIB="$R/mpistragglers.jl_amd/_build_asan/libmpiasyncpools.so" \
  python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider -k "not mpi_cpu_baseline_runs" "$@"
