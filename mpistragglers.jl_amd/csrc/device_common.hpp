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
__device__ __forceinline__ bool disarmed(const unsigned long long* go, unsigned long long seq) {
  return go && __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == seq;
}

}  // namespace dev
}  // namespace mpa
