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

// Completion publish of a task whose reply stays in this GPU's memory and is read only by later
// kernels on this GPU (the coordinator's own workers; the host reads nothing but the completion
// word): the agent-scope release makes the reply visible on the device, and the word itself goes
// out as a system-scope store, without publish_done's two system-scope L2 writebacks on every
// task's completion path.  A reply another process or device reads keeps publish_done.
__device__ __forceinline__ void publish_done_local(unsigned long long* flag, unsigned long long seq) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  drain_vm();
  __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// As publish_done_local, for a reply every byte of which its writers stored write-through
// (agent-scope relaxed stores: global_store sc1) and drained (s_waitcnt vmcnt(0)) before the
// workgroup barrier that precedes this call: there is nothing left to release, and the
// readers (the next step, after its own acquire) find the bytes past the L2s
// (MI355X_MICROARCH.md, the "sc1 stores" valid form).
__device__ __forceinline__ void publish_done_wt(unsigned long long* flag, unsigned long long seq) {
  __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// N > 1: a worker process's task also stores its completion into rank 0's GPU memory (a word
// after its reply inbox, over xGMI), where rank 0's fused tail / wait kernel polls it instead of
// the host-memory word across PCIe (round 6).  After publish_done's system-scope fence: the reply
// is visible before either word.
__device__ __forceinline__ void publish_peer(unsigned long long* flag2, unsigned long long seq) {
  if (flag2) __hip_atomic_store(flag2, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void publish_task(unsigned long long* flag, unsigned long long seq, int local) {
  if (local) publish_done_local(flag, seq);
  else publish_done(flag, seq);
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

// A device-armed task of a worker process is launched before rank 0 posts
// it and waits in-kernel for its doorbell: a word in this GPU's fine-grained message slot
// that rank 0's exchange / epoch kernel stores over xGMI after the message (release, system
// scope).  Thread 0 of every workgroup polls it with relaxed system-scope loads (they bypass
// the caches and invalidate nothing: an acquiring poll invalidated L2 at every load and, on a
// GPU shared with rank 0 in a one-GPU rehearsal, slowed its kernels 1.8x) until it reaches the
// task's seq, with or without kCancelBit (a task its server cancelled runs and then neither
// writes nor publishes, as its go word says), then acquires once: the message the store
// released is visible to the workgroup after the barrier.  Bounded by spin_ticks: error bit
// 64 and no work.  Call with the whole workgroup.
__device__ __forceinline__ bool wait_door(const unsigned long long* door, unsigned long long seq,
                                          unsigned long long spin_ticks, unsigned* err) {
  __shared__ int s_door_ok;
  if (threadIdx.x == 0) {
    const unsigned long long t0 = rt_now();
    int ok = 1;
    for (unsigned k = 0;
         (__hip_atomic_load(door, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & ~kCancelBit) < seq; ++k) {
      __builtin_amdgcn_s_sleep(2);
      if ((k & 255) == 255 && rt_now() - t0 > spin_ticks) {
        __hip_atomic_fetch_or(err, 64u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope, once
    s_door_ok = ok;
  }
  __syncthreads();
  return s_door_ok != 0;
}

}  // namespace dev
}  // namespace mpa
