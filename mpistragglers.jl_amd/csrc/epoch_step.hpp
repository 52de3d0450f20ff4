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

// Every pointer the step touches is global memory (this GPU's, a peer's or pinned host memory),
// and its loads and stores go through address space 1 as global_* instructions.  Generic (flat)
// ones also count against lgkmcnt and may alias LDS: with the pre-armed head's arguments staged
// in LDS the compiler re-read each argument after every flat store and waited for every flat load
// before it (c1's head step paid a memory round trip per chunk).
#define MPA_GLOBAL __attribute__((address_space(1)))
typedef unsigned SysU4 __attribute__((ext_vector_type(4)));
typedef unsigned SysU2 __attribute__((ext_vector_type(2)));
template <typename U>
__device__ __forceinline__ U gld(const void* p) {
  return *(const MPA_GLOBAL U*)p;
}
template <typename U>
__device__ __forceinline__ void gst(void* p, U v) {
  *(MPA_GLOBAL U*)p = v;
}

template <typename T, int V>
__device__ __forceinline__ EVec<T, V> eld(const T* p) {
  if constexpr (V * sizeof(T) == 16) {
    return __builtin_bit_cast(EVec<T, V>, gld<SysU4>(p));
  } else if constexpr (V * sizeof(T) == 8 && V > 1) {
    return __builtin_bit_cast(EVec<T, V>, gld<SysU2>(p));
  } else if constexpr (V * sizeof(T) == 32) {
    struct U2 {
      SysU4 a, b;
    };
    return __builtin_bit_cast(EVec<T, V>, (U2{gld<SysU4>(p), gld<SysU4>(reinterpret_cast<const SysU4*>(p) + 1)}));
  } else {
    EVec<T, V> r;
#pragma unroll
    for (int e = 0; e < V; ++e) r.v[e] = gld<T>(p + e);
    return r;
  }
}
template <typename T, int V>
__device__ __forceinline__ void est(T* p, const EVec<T, V>& v) {
  if constexpr (V * sizeof(T) == 16) {
    gst<SysU4>(p, __builtin_bit_cast(SysU4, v));
  } else if constexpr (V * sizeof(T) == 8 && V > 1) {
    gst<SysU2>(p, __builtin_bit_cast(SysU2, v));
  } else if constexpr (V * sizeof(T) == 32) {
    struct U2 {
      SysU4 a, b;
    };
    const U2 u = __builtin_bit_cast(U2, v);
    gst<SysU4>(p, u.a);
    gst<SysU4>(reinterpret_cast<SysU4*>(p) + 1, u.b);
  } else {
#pragma unroll
    for (int e = 0; e < V; ++e) gst<T>(p + e, v.v[e]);
  }
}

// V bf16 message elements as ONE store / load: 16 B at V = 8, 8 B at V = 4, 4 B at V = 2
// (epoch_width guarantees the alignment), element stores otherwise.  A remote worker's message slot is
// fine-grained memory of another GPU: element stores reached it as 2-byte partial writes
// (c5 at N = 2 moved 22 GB/s, at N = 8 2.3 GB/s).
template <int V>
using H16 = EVec<uint16_t, V>;
template <int V>
__device__ __forceinline__ void st_bf16(uint16_t* p, const H16<V> h) {
  if constexpr (V == 8) {
    gst<SysU4>(p, __builtin_bit_cast(SysU4, h));
  } else if constexpr (V == 4) {
    gst<SysU2>(p, __builtin_bit_cast(SysU2, h));
  } else if constexpr (V == 2) {
    gst<unsigned>(p, __builtin_bit_cast(unsigned, h));
  } else {
#pragma unroll
    for (int e = 0; e < V; ++e) gst<uint16_t>(p + e, h.v[e]);
  }
}
template <int V>
__device__ __forceinline__ H16<V> ld_bf16(const uint16_t* p) {
  if constexpr (V == 8) {
    return __builtin_bit_cast(H16<V>, gld<SysU4>(p));
  } else if constexpr (V == 4) {
    return __builtin_bit_cast(H16<V>, gld<SysU2>(p));
  } else if constexpr (V == 2) {
    return __builtin_bit_cast(H16<V>, gld<unsigned>(p));
  } else {
    H16<V> h;
#pragma unroll
    for (int e = 0; e < V; ++e) h.v[e] = gld<uint16_t>(p + e);
    return h;
  }
}

// System-scope write-through stores (sc0 sc1: the bytes go to memory instead of sitting dirty in
// this XCD's L2) of the messages other processes read.  Once every storing wave has drained
// them (s_waitcnt vmcnt(0)) they are visible at system scope, so the doorbell behind them needs
// no L2 writeback: a system-scope release fence in every workgroup wrote back each XCD's whole
// L2 (the recvbuf, x and mirror stores of the step too) before the doorbells could ring.
__device__ __forceinline__ void st_sys(void* p, uint4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(__builtin_bit_cast(SysU4, v)) : "memory");
}
__device__ __forceinline__ void st_sys(void* p, uint2 v) {
  asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(__builtin_bit_cast(SysU2, v)) : "memory");
}
__device__ __forceinline__ void st_sys(void* p, unsigned v) {
  asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sys(void* p, unsigned short v) {
  asm volatile("global_store_short %0, %1, off sc0 sc1" ::"v"(p), "v"(unsigned(v)) : "memory");
}
template <typename T, int V>
__device__ __forceinline__ void est_sys(T* p, const EVec<T, V>& v) {
  if constexpr (V * sizeof(T) == 16) {
    st_sys(p, __builtin_bit_cast(uint4, v));
  } else if constexpr (V * sizeof(T) == 8) {
    st_sys(p, __builtin_bit_cast(uint2, v));
  } else if constexpr (V * sizeof(T) == 32) {
    struct U2 {
      uint4 a, b;
    };
    const U2 u = __builtin_bit_cast(U2, v);
    st_sys(p, u.a);
    st_sys(reinterpret_cast<uint4*>(p) + 1, u.b);
  } else {
    static_assert(V * sizeof(T) == 4, "4-, 8-, 16- or 32-B vectors");
    st_sys(p, __builtin_bit_cast(unsigned, v));
  }
}
template <int V>
__device__ __forceinline__ void st_bf16_sys(uint16_t* p, const H16<V> h) {
  if constexpr (V == 8) {
    st_sys(p, __builtin_bit_cast(uint4, h));
  } else if constexpr (V == 4) {
    st_sys(p, __builtin_bit_cast(uint2, h));
  } else if constexpr (V == 2) {
    st_sys(p, __builtin_bit_cast(unsigned, h));
  } else {
#pragma unroll
    for (int e = 0; e < V; ++e) st_sys(p + e, h.v[e]);
  }
}

// relaxed agent-scope element store / load: write-through to the coherence point, visible to
// workgroups on other XCDs without an L2 writeback / invalidate (the fused head's messages)
template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) {
  using U = typename std::conditional<sizeof(T) == 8, unsigned long long, unsigned>::type;
  __hip_atomic_store((MPA_GLOBAL U*)p, __builtin_bit_cast(U, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
  using U = typename std::conditional<sizeof(T) == 8, unsigned long long, unsigned>::type;
  return __builtin_bit_cast(T, __hip_atomic_load((const MPA_GLOBAL U*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Vectors jv = first, first + stride, ... of V elements (16-B vectors when every pointer
// allows it).  Every chunk load is issued unconditionally before any arithmetic (chunks past
// n read x, a valid address, and are ignored): a load under a branch made the compiler wait
// for each one in turn.
// WT: the dispatch copies are stored write-through (st_agent; the fused head, not bf16 messages)
// BF16 = false: the caller never passes bf16 messages or a mirror (the fused tail / head of the
// least-squares launch, transport_hip.cpp tail_fits / fused_head), so that code is left out
template <typename T, int V, bool WT = false, bool BF16 = true>
__device__ __forceinline__ void epoch_elems(const EpochArgs& a, int64_t first, int64_t stride) {
  T* recv = reinterpret_cast<T*>(a.recv);
  T* x = static_cast<T*>(a.x);
  const int64_t nv = a.elems / V;
  // chunks past n load from pad: x's address, hidden from the compiler -- a load it could
  // identify with the iterate's own it replaced by a copy of that value, which waited for the
  // iterate's load before the chunks' loads were issued (two memory round trips, not one)
  const T* pad = x;
  asm volatile("" : "+v"(pad));
  for (int64_t jv = first; jv < nv; jv += stride) {
    const int64_t j = jv * V;
    EVec<T, V> v = eld<T, V>(x + j);
    EVec<T, V> c[kMaxEpochChunks];
#pragma unroll
    for (int i = 0; i < kMaxEpochChunks; ++i) {
      const T* src = i < a.n ? (a.hsrc[i] ? reinterpret_cast<const T*>(a.hsrc[i]) : recv + int64_t(i) * a.elems) : pad;
      c[i] = eld<T, V>(src + j);
    }
#pragma unroll
    for (int i = 0; i < kMaxEpochChunks; ++i)
      if (i < a.n && a.hsrc[i]) est<T, V>(recv + int64_t(i) * a.elems + j, c[i]);
    for (int d = 0; d < a.ndst0; ++d) {  // held re-dispatches: the message before the update
      if (BF16 && a.msg_bf16) {
        st_bf16<V>(reinterpret_cast<uint16_t*>(a.dst0[d]) + j, ld_bf16<V>(a.mirror + j));
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
    if (BF16 && a.msg_bf16) {  // the message is the bf16 mirror (batched variant): a.mirror != NULL
      H16<V> h;
      if (a.update) {
#pragma unroll
        for (int e = 0; e < V; ++e) h.v[e] = f32_to_bf16_rne(float(v.v[e]));
        st_bf16<V>(a.mirror + j, h);
      } else {
        h = ld_bf16<V>(a.mirror + j);
      }
      for (int d = 0; d < a.ndst; ++d) {
        if ((a.dst_sys >> d) & 1u) st_bf16_sys<V>(reinterpret_cast<uint16_t*>(a.dst[d]) + j, h);
        else st_bf16<V>(reinterpret_cast<uint16_t*>(a.dst[d]) + j, h);
      }
    } else {
      if (BF16 && a.update && a.mirror) {
        H16<V> h;
#pragma unroll
        for (int e = 0; e < V; ++e) h.v[e] = f32_to_bf16_rne(float(v.v[e]));
        st_bf16<V>(a.mirror + j, h);
      }
      for (int d = 0; d < a.ndst; ++d) {
        if constexpr (WT) {
#pragma unroll
          for (int e = 0; e < V; ++e) st_agent(reinterpret_cast<T*>(a.dst[d]) + j + e, v.v[e]);
        } else {
          if ((a.dst_sys >> d) & 1u) est_sys<T, V>(reinterpret_cast<T*>(a.dst[d]) + j, v);
          else est<T, V>(reinterpret_cast<T*>(a.dst[d]) + j, v);
        }
      }
    }
  }
}

}  // namespace dev
}  // namespace mpa
