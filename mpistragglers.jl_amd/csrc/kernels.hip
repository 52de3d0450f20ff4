// gfx950 (CDNA4) kernels of the asyncmap! hot path.
//
//   (lsq_grad_kernel, the worker compute, lives in lsq_kernel.hip)
//   exchange_kernel   the reference's byte copies `isendbufs[i] .= sendbuf` (:130,:178) and
//                     `recvbufs[i] .= irecvbufs[i]` (:108,:167,:216), batched per flush
//   kmap_task_kernel  the reference's test worker programs (test/kmap1.jl, test/kmap2.jl)
//   aggregate_kernel  coordinator consumption of fresh chunks (iterative_example.jl:41-46)
//   generate_kernel   Philox4x32-10 synthetic data, bit-identical to oracle/philox.h
//
// Completion protocol (every worker task kernel): the reply chunk is stored, released at
// agent scope, and the LAST writer publishes `seq` into the worker's host-pinned flag with
// a system-scope release; the coordinator thread polls that word (MPI.Test!/Waitany!).
#include <hip/hip_runtime.h>

#include "device_common.hpp"
#include "epoch_step.hpp"
#include "kernels.hpp"
#include "mpiasyncpools.h"

namespace mpa {

namespace {

using namespace dev;

// ---------------------------------------------------------------------------------------
__device__ void block_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {
  if (n == 8 && ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 7u) == 0) {
    // one word, copied untorn (a doorbell value staged as a pre-armed task's go word)
    if (threadIdx.x == 0)
      *reinterpret_cast<unsigned long long*>(dst) =
          __hip_atomic_load(reinterpret_cast<const unsigned long long*>(src), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15u) == 0) {
    const uint64_t nv = n >> 4;
    uint4* d = reinterpret_cast<uint4*>(dst);
    const uint4* s = reinterpret_cast<const uint4*>(src);
    for (uint64_t j = threadIdx.x; j < nv; j += blockDim.x) d[j] = s[j];
    for (uint64_t j = (nv << 4) + threadIdx.x; j < n; j += blockDim.x) dst[j] = src[j];
  } else {
    for (uint64_t j = threadIdx.x; j < n; j += blockDim.x) dst[j] = src[j];
  }
}

__global__ void __launch_bounds__(kThreads) exchange_kernel(ExchangeArgs a) {
  const int b = blockIdx.x;
  int i = 0;  // copy item of this block (uniform scan)
  while (i + 1 < a.ncopy && b >= a.block0[i + 1]) ++i;
  if (a.ncopy > 0) {
    const CopyItem& c = a.c[i];
    const uint64_t off = uint64_t(b - a.block0[i]) * a.part;
    if (off < c.bytes) {
      const uint64_t len = (c.bytes - off) < a.part ? (c.bytes - off) : a.part;
      block_copy(c.dst + off, c.src + off, len);
    }
  }
  if (a.ndoor == 0) return;
  // every block's copies drained and released at system scope (the mailboxes are host
  // memory read by another GPU), then the last block to arrive rings the doorbells
  __shared__ unsigned s_last;
  drain_vm();
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old - a.ticket_base) == gridDim.x - 1;
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      for (int d = 0; d < a.ndoor; ++d)
        __hip_atomic_store(a.door[d], a.doorval[d], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) wait_words_kernel(WaitWordsArgs a) {
  const int j = threadIdx.x;
  bool ok = j >= a.n;
  const unsigned long long t0 = rt_now();
  for (unsigned k = 0;; ++k) {
    if (!ok) ok = __hip_atomic_load(a.word[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= a.target[j];
    if (__builtin_amdgcn_ballot_w64(!ok) == 0ull) break;  // every word reached (exit for the whole wave)
    __builtin_amdgcn_s_sleep(2);
    if ((k & 63) == 63 && rt_now() - t0 > a.spin_ticks) {  // bounded: report and return
      if (j == 0) __hip_atomic_fetch_or(a.err, 32u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the replies the remote tasks released
}

// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) kmap_task_kernel(KmapArgs a) {
  if (a.stamp && threadIdx.x == 0) __hip_atomic_store(a.stamp, rt_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (a.kind == MPA_TASK_ECHO) {
    const uint64_t m = a.sl < a.rl ? a.sl : a.rl;
    for (uint64_t j = threadIdx.x; j < a.rl; j += blockDim.x) a.out[j] = j < m ? a.x[j] : uint8_t(0);
  } else if (threadIdx.x == 0) {
    double v[3] = {a.rank, double(a.pub.seq), 0.0};  // t == tasks served (kmap2.jl:82-84)
    uint8_t* vb = reinterpret_cast<uint8_t*>(v);
    if (a.kind == MPA_TASK_KMAP2) {
      for (uint64_t j = 0; j < 8 && j < a.sl; ++j) vb[16 + j] = a.x[j];  // epoch = recvbuf[1]
    }
    const uint64_t m = a.kind == MPA_TASK_KMAP1 ? 8 : 24;
    for (uint64_t j = 0; j < a.rl; ++j) a.out[j] = j < m ? vb[j] : uint8_t(0);
  }
  drain_vm();
  __syncthreads();
  if (a.stamp && threadIdx.x == 0) __hip_atomic_store(a.stamp + 1, rt_now(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (threadIdx.x == 0) publish_task(a.pub.flag, a.pub.seq, a.pub_local);
}

__global__ void __launch_bounds__(64) clock_probe_kernel(unsigned long long* out) {
  if (threadIdx.x == 0) __hip_atomic_store(out, rt_now(), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------------------

template <typename T>
__global__ void __launch_bounds__(kThreads) aggregate_kernel(AggregateArgs a) {
  const T* c = static_cast<const T*>(a.chunks);
  T* out = static_cast<T*>(a.out);
  for (int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < a.elems;
       j += int64_t(gridDim.x) * blockDim.x) {
    // explicit fused multiply-adds: the arithmetic may not depend on how the compiler
    // contracts the loop, so the fused epoch kernel below rounds identically
    double s = 0.0;
    for (int64_t i = 0; i < a.n; ++i)
      if (a.w[i] != 0.0) s = __builtin_fma(a.w[i], double(c[i * a.stride + j]), s);
    const T v = a.update ? T(__builtin_fma(-a.eta, s, double(out[j]))) : T(s);
    out[j] = v;
    if (a.mirror) a.mirror[j] = f32_to_bf16_rne(float(v));
  }
}

// ---------------------------------------------------------------------------------------
// The fused coordinator epoch step (EpochArgs, epoch_step.hpp): one thread per V elements,
// then the doorbells of remote workers.  Same arithmetic as aggregate_kernel (fp64 sum in
// chunk order), so the fused and unfused loops produce identical iterates.
template <typename T, int V>
__global__ void __launch_bounds__(kThreads) epoch_kernel(EpochArgs a) {
  epoch_elems<T, V>(a, int64_t(blockIdx.x) * blockDim.x + threadIdx.x, int64_t(gridDim.x) * blockDim.x);
  if (a.ndoor == 0) return;
  // every block's message stores drained, then the last block to arrive rings the doorbells.
  // The remote messages went out write-through at system scope (EpochArgs::dst_sys): drained,
  // they are visible to the other processes, and no block writes back its L2.  sys_fence
  // (MPA_MSG_WT=0): plain stores, released at system scope by every block, as exchange_kernel.
  __shared__ unsigned s_last;
  drain_vm();
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.sys_fence) {
      __threadfence_system();
      drain_vm();
    }
    const unsigned old = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old - a.ticket_base) == gridDim.x - 1;
    if (s_last) {
      if (a.sys_fence) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        for (int d = 0; d < a.ndoor; ++d)
          __hip_atomic_store(a.door[d], a.doorval[d], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        for (int d = 0; d < a.ndoor; ++d)
          __hip_atomic_store(a.door[d], a.doorval[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = uint64_t(0xD2511F53u) * c[0];
    const uint64_t p1 = uint64_t(0xCD9E8D57u) * c[2];
    const uint32_t n0 = uint32_t(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = uint32_t(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0; c[1] = uint32_t(p1); c[2] = n2; c[3] = uint32_t(p0);
  }
}

__device__ __forceinline__ float unit_f32(uint32_t w) {
  return float(int32_t(w >> 8) - 8388608) * (1.0f / 8388608.0f);
}

__global__ void __launch_bounds__(kThreads) generate_kernel(void* out, int dtype, uint64_t seed, uint32_t stream,
                                                           uint64_t e0, int64_t count, double scale) {
  const uint64_t q0 = e0 >> 2, q1 = (e0 + uint64_t(count) + 3) >> 2;
  const float sf = float(scale);
  for (uint64_t q = q0 + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; q < q1;
       q += uint64_t(gridDim.x) * blockDim.x) {
    uint32_t c[4] = {uint32_t(q), uint32_t(q >> 32), stream, 0u};
    philox4x32_10(c, uint32_t(seed), uint32_t(seed >> 32));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t e = q * 4 + uint64_t(j);
      if (e < e0 || e >= e0 + uint64_t(count)) continue;
      const uint64_t k = e - e0;
      if (dtype == MPA_F64) {
        static_cast<double*>(out)[k] = double(unit_f32(c[j])) * scale;
      } else if (dtype == MPA_BF16) {
        static_cast<uint16_t*>(out)[k] = f32_to_bf16_rne(unit_f32(c[j]) * sf);
      } else {
        static_cast<float*>(out)[k] = unit_f32(c[j]) * sf;
      }
    }
  }
}

// Measured HBM read ceiling for the roofline context (mpa_read_bandwidth): a streaming
// read of `n16` 16-B vectors.  Workgroup b reads one contiguous 1/grid of the buffer, 16 KiB
// per step (four non-temporal 16-B loads in flight per thread, each wave-instruction 1 KiB
// contiguous), folded into one word per workgroup (the store keeps the loads live).
__global__ void __launch_bounds__(kThreads) read_peak_kernel(const uint4* __restrict__ p, uint64_t n16,
                                                             uint32_t* __restrict__ sink) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = per * blockIdx.x, hi = lo + per < n16 ? lo + per : n16;
  uint32_t x = 0;
  uint64_t j = lo + threadIdx.x;
  for (; j + 3 * kThreads < hi; j += 4 * kThreads) {
    const u32x4 a = __builtin_nontemporal_load(q + j), b = __builtin_nontemporal_load(q + j + kThreads);
    const u32x4 c = __builtin_nontemporal_load(q + j + 2 * kThreads), d = __builtin_nontemporal_load(q + j + 3 * kThreads);
    const u32x4 v = a ^ b ^ c ^ d;  // every word used: the loads stay 16 B wide
    x ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  for (; j < hi; j += kThreads) {
    const u32x4 v = __builtin_nontemporal_load(q + j);
    x ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  x = __reduce_or_sync(0xffffffffffffffffull, x);
  if (threadIdx.x == 0) sink[blockIdx.x] = x;
}

}  // namespace

hipError_t launch_wait_words(const WaitWordsArgs& a, hipStream_t s) {
  if (a.n <= 0 || a.n > kMaxWaitWords) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wait_words_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_exchange(const ExchangeArgs& a, hipStream_t s) {
  int grid = a.block0[a.ncopy];
  if (grid == 0 && a.ndoor > 0) grid = 1;  // doorbells only
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(exchange_kernel, dim3(grid), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

__global__ void __launch_bounds__(64) door_cas_kernel(unsigned long long* door, unsigned long long expect,
                                                      unsigned long long desired, unsigned long long* old_out) {
  if (threadIdx.x != 0) return;
  unsigned long long e = expect;
  __hip_atomic_compare_exchange_strong(door, &e, desired, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(old_out, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_door_cas(unsigned long long* door, unsigned long long expect, unsigned long long desired,
                           unsigned long long* old_out, hipStream_t s) {
  hipLaunchKernelGGL(door_cas_kernel, dim3(1), dim3(64), 0, s, door, expect, desired, old_out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// A device-armed task's doorbell wait as a kernel of its own (hip_server.cpp arm, the
// default MPA_ARM_WAIT=wave): ONE wave polls the worker's device doorbell (wait_door's loop:
// relaxed system-scope loads, s_sleep, bounded, then one system-scope acquire) and exits;
// the task kernel queued behind it on the worker's stream starts when the packet processor
// moves on.  A waiting armed task holds one wave instead of its whole launch grid, so armed
// worker processes sharing a GPU with rank 0 (a one-GPU rehearsal) cannot starve the
// kernels that ring their doorbells (profiles/r03_rehearsal_n248.txt).
// A wait that times out cancels the task queued behind it: the wave stores the
// task's seq into the task's go word before it sets err bit 64, so the task -- the non-armed
// instantiation, which only checks that word -- neither writes its reply nor publishes `done`
// on a message rank 0 never posted.
__global__ void __launch_bounds__(64) door_wait_kernel(const unsigned long long* door, unsigned long long seq,
                                                       unsigned long long spin_ticks, unsigned* err,
                                                       unsigned long long* cancel, unsigned long long delay_ticks) {
  if (threadIdx.x) return;
  const unsigned long long t0 = rt_now();
  unsigned long long d = 0;
  for (unsigned k = 0; ((d = __hip_atomic_load(door, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) & ~kCancelBit) < seq;
       ++k) {
    __builtin_amdgcn_s_sleep(2);
    if ((k & 255) == 255 && rt_now() - t0 > spin_ticks) {
      __hip_atomic_store(cancel, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_fetch_or(err, 64u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      d = kCancelBit;
      break;
    }
  }
  // a delayed worker (an injected straggler, test/kmap2.jl:95's sleep between its Irecv and its
  // reply) sleeps from the moment its doorbell rang, here on the device: no host thread between
  // the ring and the task (a cancelled task -- pause / shutdown -- does not sleep)
  if (delay_ticks && !(d & kCancelBit)) {
    const unsigned long long t1 = rt_now();
    while (rt_now() - t1 < delay_ticks) __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the message the doorbell released
}

hipError_t launch_door_wait(const unsigned long long* door, unsigned long long seq, unsigned long long spin_ticks,
                            unsigned* err, unsigned long long* cancel, unsigned long long delay_ticks, hipStream_t s) {
  if (!door || !err || !cancel) return hipErrorInvalidValue;
  hipLaunchKernelGGL(door_wait_kernel, dim3(1), dim3(64), 0, s, door, seq, spin_ticks, err, cancel, delay_ticks);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Straggler emulation: the reference worker sleeps rand() between its Irecv and
// its reply (examples/iterative_example.jl:74, test/kmap2.jl:95).  A delayed worker of the
// coordinator's process waits on its worker's stream, ahead of the task, in this one-wave
// kernel until an ABSOLUTE deadline on the GPU's constant 100 MHz clock (the host's post time +
// the delay, mapped through the clock calibration, HipComm::device_deadline): when the stream
// reaches it does not matter, no host thread has to wake up on time, one wave holds no CU anyone
// else needs.  Bounded (err bit 256).  (A device-armed worker of another process sleeps inside
// its door_wait_kernel instead, from its doorbell.)
__global__ void __launch_bounds__(64) deadline_kernel(unsigned long long deadline, unsigned long long bound,
                                                       unsigned* err) {
  if (threadIdx.x) return;
  const unsigned long long t0 = rt_now();
  for (;;) {
    const unsigned long long t = rt_now();
    if (t >= deadline) break;
    if (t - t0 > bound) {
      __hip_atomic_fetch_or(err, 256u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

hipError_t launch_deadline(unsigned long long deadline, unsigned long long bound, unsigned* err, hipStream_t s) {
  hipLaunchKernelGGL(deadline_kernel, dim3(1), dim3(64), 0, s, deadline, bound, err);
  return hipGetLastError();
}

hipError_t launch_clock_probe(unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, s, out);
  return hipGetLastError();
}

hipError_t launch_kmap(const KmapArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(kmap_task_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_aggregate(int dtype, const AggregateArgs& a, hipStream_t s) {
  const int grid = int((a.elems + kThreads - 1) / kThreads) < 1024 ? int((a.elems + kThreads - 1) / kThreads) : 1024;
  if (grid <= 0) return hipSuccess;
  if (dtype == MPA_F32) hipLaunchKernelGGL(aggregate_kernel<float>, dim3(grid), dim3(kThreads), 0, s, a);
  else if (dtype == MPA_F64) hipLaunchKernelGGL(aggregate_kernel<double>, dim3(grid), dim3(kThreads), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// Elements per thread of the epoch step: 16-B vectors of the iterate (4 fp32 / 2 fp64) when
// the element count and every pointer the kernel touches allow it; fp32 with bf16 messages
// (the batched variant) up to 8, so each message store is one 16-B vector (4: 8 B).  A large
// step (c5: 131072 elements) then narrows its vectors until the grid covers the chip
// (kEpochMinGrid workgroups, one per CU), down to 8-B accesses: at 8 elements per thread c5's
// step ran on 64 workgroups.
#ifndef MPA_EPOCH_MIN_GRID
#define MPA_EPOCH_MIN_GRID 256
#endif
static int epoch_width_max(int dtype, const EpochArgs& a);
int epoch_width(int dtype, const EpochArgs& a) {
  int v = epoch_width_max(dtype, a);
  const int floor_v = dtype == MPA_F64 ? 1 : 2;  // keep 8-B accesses
  // (a small step -- c1-c4's iterate of 64-2048 elements -- keeps its widest vectors: one or a
  // few workgroups either way)
  while (v > floor_v && a.elems / v / kThreads < MPA_EPOCH_MIN_GRID && a.elems / v / kThreads >= 32) v /= 2;
  return v;
}

static int epoch_width_max(int dtype, const EpochArgs& a) {
  uintptr_t m = reinterpret_cast<uintptr_t>(a.recv) | reinterpret_cast<uintptr_t>(a.x);
  for (int i = 0; i < a.n; ++i)
    m |= reinterpret_cast<uintptr_t>(a.hsrc[i]) | reinterpret_cast<uintptr_t>(a.hsrc2[i]);
  uintptr_t mb = reinterpret_cast<uintptr_t>(a.mirror);  // bf16 stores
  for (int d = 0; d < a.ndst; ++d) (a.msg_bf16 ? mb : m) |= reinterpret_cast<uintptr_t>(a.dst[d]);
  for (int d = 0; d < a.ndst0; ++d) (a.msg_bf16 ? mb : m) |= reinterpret_cast<uintptr_t>(a.dst0[d]);
  if (dtype == MPA_F64) return a.elems % 2 == 0 && (m & 15u) == 0 && (mb & 3u) == 0 ? 2 : 1;
  if (a.msg_bf16 && a.elems % 8 == 0 && ((m | mb) & 15u) == 0) return 8;
  return a.elems % 4 == 0 && (m & 15u) == 0 && (mb & 7u) == 0 ? 4 : 1;
}

bool epoch_vec(int dtype, const EpochArgs& a) { return epoch_width_max(dtype, a) > 1; }

int epoch_grid(int dtype, const EpochArgs& a) {
  const int V = epoch_width(dtype, a);
  const int64_t g = (a.elems / V + kThreads - 1) / kThreads;
  return int(g < 1 ? 1 : g > 1024 ? 1024 : g);
}

hipError_t launch_epoch(int dtype, const EpochArgs& a, hipStream_t s) {
  const int grid = epoch_grid(dtype, a);
  const int width = epoch_width(dtype, a);
  const bool vec = width > 1;
  if (dtype == MPA_F32) {
    if (width == 8) hipLaunchKernelGGL((epoch_kernel<float, 8>), dim3(grid), dim3(kThreads), 0, s, a);
    else if (width == 4) hipLaunchKernelGGL((epoch_kernel<float, 4>), dim3(grid), dim3(kThreads), 0, s, a);
    else if (width == 2) hipLaunchKernelGGL((epoch_kernel<float, 2>), dim3(grid), dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((epoch_kernel<float, 1>), dim3(grid), dim3(kThreads), 0, s, a);
  } else if (dtype == MPA_F64) {
    if (vec) hipLaunchKernelGGL((epoch_kernel<double, 2>), dim3(grid), dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((epoch_kernel<double, 1>), dim3(grid), dim3(kThreads), 0, s, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_generate(void* out, int dtype, uint64_t seed, uint32_t stream, uint64_t e0, int64_t count,
                           double scale, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  const uint64_t quads = ((e0 + uint64_t(count) + 3) >> 2) - (e0 >> 2);
  const uint64_t want = (quads + kThreads - 1) / kThreads;
  const int grid = int(want < 8192 ? want : 8192);
  hipLaunchKernelGGL(generate_kernel, dim3(grid), dim3(kThreads), 0, s, out, dtype, seed, stream, e0, count, scale);
  return hipGetLastError();
}

hipError_t launch_read_peak(const void* p, uint64_t bytes, int grid, uint32_t* sink, hipStream_t s) {
  hipLaunchKernelGGL(read_peak_kernel, dim3(grid), dim3(kThreads), 0, s, static_cast<const uint4*>(p), bytes / 16, sink);
  return hipGetLastError();
}

}  // namespace mpa
