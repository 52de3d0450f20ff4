// Device helpers of the fp32 / fp64 least-squares kernels (lsq_kernel.hip, the narrow
// single pass; lsqw_kernel.hip, the wide two passes): 16-B vector loads, the DPP wave sum,
// and the write-through partial hand-off of the reduction trees.
#pragma once
#include <hip/hip_runtime.h>

#include "device_common.hpp"

namespace mpa {
namespace dev {

template <typename T>
struct VecOf;
template <>
struct VecOf<float> {
  typedef float type __attribute__((ext_vector_type(4)));
};
template <>
struct VecOf<double> {
  typedef double type __attribute__((ext_vector_type(2)));
};

template <typename T, bool NT>
__device__ __forceinline__ Pack<T> ld16(const Pack<T>* p) {
  using V = typename VecOf<T>::type;
  V v;
  if constexpr (NT) v = __builtin_nontemporal_load(reinterpret_cast<const V*>(p));
  else v = *reinterpret_cast<const V*>(p);
  Pack<T> r;
#pragma unroll
  for (int e = 0; e < Pack<T>::E; ++e) r.v[e] = v[e];
  return r;
}

// DPP lane move with zero for lanes whose source is out of the row / masked row
template <int CTRL, int RMASK>
__device__ __forceinline__ float dpp_f32(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, RMASK, 0xF, false));
}
template <int CTRL, int RMASK>
__device__ __forceinline__ double dpp_f64(double x) {
  const long long u = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, int(u), CTRL, RMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, int(u >> 32), CTRL, RMASK, 0xF, false);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

__device__ __forceinline__ float dpp_add_f32(float v) {
  // 64-lane sum: quad_perm [1,0,3,2], [2,3,0,1], row_shr 4, row_shr 8 (row totals in lanes
  // 12-15 of each row), row_bcast 15 (rows 1,3), row_bcast 31 (rows 2,3): lane 63 = total.
  v += dpp_f32<0xB1, 0xF>(v);
  v += dpp_f32<0x4E, 0xF>(v);
  v += dpp_f32<0x114, 0xF>(v);
  v += dpp_f32<0x118, 0xF>(v);
  v += dpp_f32<0x142, 0xA>(v);
  v += dpp_f32<0x143, 0xC>(v);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

__device__ __forceinline__ double dpp_add_f64(double v) {
  v += dpp_f64<0xB1, 0xF>(v);
  v += dpp_f64<0x4E, 0xF>(v);
  v += dpp_f64<0x114, 0xF>(v);
  v += dpp_f64<0x118, 0xF>(v);
  v += dpp_f64<0x142, 0xA>(v);
  v += dpp_f64<0x143, 0xC>(v);
  const long long u = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane(int(u), 63);
  const int hi = __builtin_amdgcn_readlane(int(u >> 32), 63);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

template <typename T, bool DPP>
__device__ __forceinline__ T wave_sum(T v) {
  if constexpr (DPP) {
    if constexpr (sizeof(T) == 4) return dpp_add_f32(v);
    else return dpp_add_f64(v);
  } else {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  }
}

// Slab partials move between workgroups write-through: 8-B relaxed agent-scope stores and
// loads (global_store/load_dwordx2 sc1: L1 bypassed, L2-served), so a hand-off needs no
// release / acquire fence (MI355X_MICROARCH.md §inter-workgroup visibility, the "one lane
// adds for the workgroup, the last adder loads" row): each storing wave drains its stores
// before the workgroup barrier, one lane then adds to the group counter.
template <typename T>
__device__ __forceinline__ void st_sc1(Pack<T>* p, const Pack<T>& v) {
  struct U2 {
    unsigned long long a, b;
  };
  const U2 u = __builtin_bit_cast(U2, v);
  unsigned long long* d = reinterpret_cast<unsigned long long*>(p);
  __hip_atomic_store(d, u.a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(d + 1, u.b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ Pack<T> ld_sc1(const Pack<T>* p) {
  struct U2 {
    unsigned long long a, b;
  };
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
  U2 u;
  u.a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  u.b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_bit_cast(Pack<T>, u);
}

}  // namespace dev
}  // namespace mpa
