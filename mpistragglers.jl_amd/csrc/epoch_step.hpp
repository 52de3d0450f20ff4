// The coordinator's epoch step (EpochArgs, kernels.hpp) as a device function, shared by the
// stand-alone epoch_kernel (kernels.hip) and the fused tail of the least-squares launch
// (lsq_kernel.hip: the last task of a launch to complete runs the NEXT epoch's step, so an
// epoch of the native descent loop at nwait = n is one launch).
//
// Per element j of the iterate, in the reference's order: the pending harvest copies
// `recvbufs[i] .= irecvbufs[i]` (src/MPIAsyncPools.jl:167), the messages of held stale
// re-dispatches (:180-182, the iterate before this update), the iterate update
// x -= eta * sum_i w_i chunk_i (examples/iterative_example.jl:41-46, the fp64 sum of
// aggregate_kernel in chunk order, explicit fmas), the harvests that follow the update, and
// the dispatch copies `isendbufs[i] .= sendbuf` (:130).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "kernels.hpp"

namespace mpa {
namespace dev {

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return uint16_t((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

template <typename T, int V>
struct EVec {
  T v[V];
};
template <typename T, int V>
__device__ __forceinline__ EVec<T, V> eld(const T* p) {
  if constexpr (V * sizeof(T) == 16) {
    return __builtin_bit_cast(EVec<T, V>, *reinterpret_cast<const uint4*>(p));
  } else {
    EVec<T, V> r;
#pragma unroll
    for (int e = 0; e < V; ++e) r.v[e] = p[e];
    return r;
  }
}
template <typename T, int V>
__device__ __forceinline__ void est(T* p, const EVec<T, V>& v) {
  if constexpr (V * sizeof(T) == 16) *reinterpret_cast<uint4*>(p) = __builtin_bit_cast(uint4, v);
  else
#pragma unroll
    for (int e = 0; e < V; ++e) p[e] = v.v[e];
}

// relaxed agent-scope element store / load: write-through to the coherence point, visible to
// workgroups on other XCDs without an L2 writeback / invalidate (the fused head's messages)
template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) {
  using U = typename std::conditional<sizeof(T) == 8, unsigned long long, unsigned>::type;
  __hip_atomic_store(reinterpret_cast<U*>(p), __builtin_bit_cast(U, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
  using U = typename std::conditional<sizeof(T) == 8, unsigned long long, unsigned>::type;
  return __builtin_bit_cast(T, __hip_atomic_load(reinterpret_cast<const U*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Vectors jv = first, first + stride, ... of V elements (16-B vectors when every pointer
// allows it).  Every chunk load is issued unconditionally before any arithmetic (chunks past
// n read x, a valid address, and are ignored): a load under a branch made the compiler wait
// for each one in turn.
// WT: the dispatch copies are stored write-through (st_agent; the fused head, not bf16 messages)
template <typename T, int V, bool WT = false>
__device__ __forceinline__ void epoch_elems(const EpochArgs& a, int64_t first, int64_t stride) {
  T* recv = reinterpret_cast<T*>(a.recv);
  T* x = static_cast<T*>(a.x);
  const int64_t nv = a.elems / V;
  for (int64_t jv = first; jv < nv; jv += stride) {
    const int64_t j = jv * V;
    EVec<T, V> v = eld<T, V>(x + j);
    EVec<T, V> c[kMaxEpochChunks];
#pragma unroll
    for (int i = 0; i < kMaxEpochChunks; ++i) {
      const T* src = i < a.n ? (a.hsrc[i] ? reinterpret_cast<const T*>(a.hsrc[i]) : recv + int64_t(i) * a.elems) : x;
      c[i] = eld<T, V>(src + j);
    }
#pragma unroll
    for (int i = 0; i < kMaxEpochChunks; ++i)
      if (i < a.n && a.hsrc[i]) est<T, V>(recv + int64_t(i) * a.elems + j, c[i]);
    for (int d = 0; d < a.ndst0; ++d) {  // held re-dispatches: the message before the update
      if (a.msg_bf16) {
#pragma unroll
        for (int e = 0; e < V; ++e) reinterpret_cast<uint16_t*>(a.dst0[d])[j + e] = a.mirror[j + e];
      } else if constexpr (WT) {
#pragma unroll
        for (int e = 0; e < V; ++e) st_agent(reinterpret_cast<T*>(a.dst0[d]) + j + e, v.v[e]);
      } else {
        est<T, V>(reinterpret_cast<T*>(a.dst0[d]) + j, v);
      }
    }
    if (a.update) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        double s = 0.0;  // the fp64 sum of aggregate_kernel, in chunk order
#pragma unroll
        for (int i = 0; i < kMaxEpochChunks; ++i)
          if (i < a.n && a.w[i] != 0.0) s = __builtin_fma(a.w[i], double(c[i].v[e]), s);
        v.v[e] = T(__builtin_fma(-a.eta, s, double(v.v[e])));
      }
      est<T, V>(x + j, v);
    }
    for (int i = 0; i < a.n; ++i)
      if (a.hsrc2[i]) est<T, V>(recv + int64_t(i) * a.elems + j, eld<T, V>(reinterpret_cast<const T*>(a.hsrc2[i]) + j));
    if (a.msg_bf16) {  // the message is the bf16 mirror (batched variant): a.mirror != NULL
      uint16_t h[V];
#pragma unroll
      for (int e = 0; e < V; ++e) h[e] = a.update ? f32_to_bf16_rne(float(v.v[e])) : a.mirror[j + e];
#pragma unroll
      for (int e = 0; e < V; ++e)
        if (a.update) a.mirror[j + e] = h[e];
      for (int d = 0; d < a.ndst; ++d)
#pragma unroll
        for (int e = 0; e < V; ++e) reinterpret_cast<uint16_t*>(a.dst[d])[j + e] = h[e];
    } else {
      if (a.update && a.mirror)
#pragma unroll
        for (int e = 0; e < V; ++e) a.mirror[j + e] = f32_to_bf16_rne(float(v.v[e]));
      for (int d = 0; d < a.ndst; ++d) {
        if constexpr (WT) {
#pragma unroll
          for (int e = 0; e < V; ++e) st_agent(reinterpret_cast<T*>(a.dst[d]) + j + e, v.v[e]);
        } else {
          est<T, V>(reinterpret_cast<T*>(a.dst[d]) + j, v);
        }
      }
    }
  }
}

}  // namespace dev
}  // namespace mpa
