// Device helpers shared by the gfx950 kernels (kernels.hip, lsq_kernel.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace mpa {
namespace dev {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

// 16-byte vector of T (4 x fp32 / 2 x fp64)
template <typename T>
struct alignas(16) Pack {
  static constexpr int E = 16 / sizeof(T);
  T v[E];
};

__device__ __forceinline__ unsigned long long rt_now() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Completion publish of a worker task (MI355X_MICROARCH.md §visibility, Guideline 16 R1):
// every storing wave has drained its stores and passed a workgroup barrier; ONE lane then
// releases at agent scope (the reply chunk is read by a later kernel on this device),
// releases at system scope, and stores the task's sequence number into the worker's
// host-pinned completion word that the coordinator thread polls.
__device__ __forceinline__ void publish_done(unsigned long long* flag, unsigned long long seq) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  drain_vm();
  __threadfence_system();
  drain_vm();
  __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A pre-armed launch its server cancelled: the server's host-pinned cancel word holds the
// task's seq (set before the doorbell wait is released, cleared once the stream has
// drained, so every workgroup of the task reads the same value): return before any work.
// ONE lane per wave reads the word (a host-memory read over the bus) and broadcasts it:
// with every lane reading, a 192-workgroup task spent ~125 us in these reads (one-GPU
// N = 2 rehearsal, profiles/r02_arm_go_word.txt).  Call with every lane of the wave active.
__device__ __forceinline__ bool disarmed(const unsigned long long* go, unsigned long long seq) {
  if (!go) return false;  // kernel argument: wave-uniform
  unsigned long long v = 0;
  if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0u)
    v = __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(v)), hi = __builtin_amdgcn_readfirstlane(unsigned(v >> 32));
  return ((unsigned long long)hi << 32 | lo) == seq;
}

}  // namespace dev
}  // namespace mpa
