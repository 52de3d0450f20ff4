// Least-squares worker compute for WIDE rows (cols > 2048, fp32 / fp64): the narrow kernel
// (lsq_kernel.hip) keeps x and g of a whole row in a wave's registers, which caps a row at
// 2048 columns; the reference's worker has no such cap (examples/iterative_example.jl:74
// computes on whatever the message holds).  Two passes, A read twice:
//   pass 1  r = A x - b       a wave per row: 16-B vectors of the row against x (read
//                             through the caches), DPP wave sum, r[row] = dot - b[row]
//   pass 2  g = A^T r         workgroup (slice s, row group q): 2048 columns of g in the
//                             lane registers, g += r[row] a[row, slice] over the group's rows;
//                             the 4 waves summed in LDS in wave order, the groups of a slice
//                             by a fan-in-8 tree of write-through partials (the last arriver
//                             carries, nothing waits); the last slice publishes completion
// Deterministic: fixed summation orders, no float atomics.  Both passes honour a pre-armed
// task's cancel word (`go`) like the narrow kernel.
#include <hip/hip_runtime.h>

#include "device_common.hpp"
#include "kernels.hpp"
#include "lsq_common.hpp"
#include "mpiasyncpools.h"

namespace mpa {
namespace {

using namespace dev;

constexpr int kUnroll = 4;  // 16-B vectors per lane in flight in pass 1

__device__ __forceinline__ float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }

template <typename T>
__device__ __forceinline__ Pack<T> x_vec(const T* __restrict__ x, int v, int cols) {
  constexpr int E = Pack<T>::E;
  Pack<T> p;
  if ((v + 1) * E <= cols) {
    p = *reinterpret_cast<const Pack<T>*>(x + size_t(v) * E);
  } else {  // the row's last, partial vector: x ends at cols (A's padding is multiplied by 0)
#pragma unroll
    for (int e = 0; e < E; ++e) p.v[e] = v * E + e < cols ? x[size_t(v) * E + e] : T(0);
  }
  return p;
}

template <typename T, bool ARMED>
__global__ void __launch_bounds__(kThreads) lsqw_resid_kernel(LsqBatch batch) {
  using P = Pack<T>;
  constexpr int E = P::E;
  int ti = 0;
  while (ti + 1 < batch.ntasks && int(blockIdx.x) >= batch.block0[ti + 1]) ++ti;
  const LsqTask& a = batch.t[ti];
  const int blk = int(blockIdx.x) - batch.block0[ti];
  if constexpr (ARMED)  // device-armed (pass 2 follows on the stream)
    if (!wait_door(a.door, a.seq, batch.spin_ticks, batch.err)) return;
  if (disarmed(a.go, a.seq)) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
  const T* __restrict__ A = static_cast<const T*>(a.A);
  const T* __restrict__ bv = static_cast<const T*>(a.b);
  const T* __restrict__ xv = static_cast<const T*>(a.x);
  T* __restrict__ r = static_cast<T*>(a.r);
  const int cols = a.cols;
  const int nvec = (cols + E - 1) / E;
  const int64_t stride = int64_t(a.grid) * kWaves;
  for (int64_t row = int64_t(blk) * kWaves + wave; row < a.rows; row += stride) {
    const P* ar = reinterpret_cast<const P*>(A + row * a.lda);
    T s = T(0);
    for (int v0 = lane; v0 < nvec; v0 += 64 * kUnroll) {
      P av[kUnroll], xr[kUnroll];
#pragma unroll
      for (int k = 0; k < kUnroll; ++k) {  // all loads first; vectors past the row clamp
        const int v = v0 + 64 * k;
        const int vc = v < nvec ? v : nvec - 1;
        av[k] = ld16<T, true>(ar + vc);
        xr[k] = x_vec<T>(xv, vc, cols);
      }
#pragma unroll
      for (int k = 0; k < kUnroll; ++k)
        if (v0 + 64 * k < nvec)
#pragma unroll
          for (int e = 0; e < E; ++e) s = fma_t(av[k].v[e], xr[k].v[e], s);
    }
    s = wave_sum<T, true>(s);
    if (lane == 0) r[row] = s - bv[row];
  }
}

// the task of a pass-2 block: blocks of task t = nslice_t * grid2_t, in task order
__device__ __forceinline__ int pass2_task(const LsqBatch& b, int bx, int* base) {
  int ti = 0, b0 = 0;
  for (; ti + 1 < b.ntasks; ++ti) {
    const int nb = (b.t[ti].cols + kLsqWideSlice - 1) / kLsqWideSlice * b.t[ti].grid2;
    if (bx < b0 + nb) break;
    b0 += nb;
  }
  *base = b0;
  return ti;
}

template <typename T, int VPL, int RB>
__global__ void __launch_bounds__(kThreads) lsqw_grad_kernel(LsqBatch batch) {
  using P = Pack<T>;
  constexpr int E = P::E;
  constexpr int S = VPL * 64;  // 16-B vectors of a slice
  static_assert(S * E == kLsqWideSlice, "a slice is kLsqWideSlice columns");
  __shared__ P red[S];
  __shared__ unsigned s_ticket;
  int base = 0;
  const int ti = pass2_task(batch, int(blockIdx.x), &base);
  const LsqTask& a = batch.t[ti];
  if (disarmed(a.go, a.seq)) return;
  const int nslice = (a.cols + kLsqWideSlice - 1) / kLsqWideSlice;
  const int blk2 = int(blockIdx.x) - base;
  const int sl = blk2 % nslice, q = blk2 / nslice, ng = a.grid2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t lo = a.rows * q / ng, hi = a.rows * (q + 1) / ng;
  const T* __restrict__ A = static_cast<const T*>(a.A) + size_t(sl) * kLsqWideSlice;
  const T* __restrict__ r = static_cast<const T*>(a.r);
  const int c0 = sl * kLsqWideSlice;

  bool vok[VPL];
  P g[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    vok[v] = c0 + (v * 64 + lane) * E < a.cols;
#pragma unroll
    for (int e = 0; e < E; ++e) g[v].v[e] = T(0);
  }
  for (int64_t row = lo + int64_t(wave) * RB; row < hi; row += int64_t(kWaves) * RB) {
    P d[RB][VPL];
    T rr[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {  // rows past the group clamp and weigh 0
      const bool ok = row + rb < hi;
      const int64_t rc = ok ? row + rb : row;
      rr[rb] = ok ? r[rc] : T(0);
      const P* ar = reinterpret_cast<const P*>(A + rc * a.lda);
#pragma unroll
      for (int v = 0; v < VPL; ++v) d[rb][v] = ld16<T, true>(ar + (vok[v] ? v * 64 + lane : 0));
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int v = 0; v < VPL; ++v)
#pragma unroll
        for (int e = 0; e < E; ++e) g[v].v[e] = fma_t(rr[rb], d[rb][v].v[e], g[v].v[e]);
  }
  // workgroup partial, waves added in fixed order
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    if (wave == w) {
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        P& dst = red[v * 64 + lane];
        if (w == 0) {
          dst = g[v];
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e) dst.v[e] += g[v].v[e];
        }
      }
    }
    __syncthreads();
  }
  // groups of the slice: fan-in-8 tree (lsq_kernel.hip's, per slice)
  constexpr unsigned F = kLsqFanIn;
  P* __restrict__ slab = static_cast<P*>(a.slab) + size_t(sl) * kLsqWideMaxGroups * S;
  uint32_t* __restrict__ ctr = a.wctr + sl * kLsqWideCtrPerSlice;
  T* __restrict__ out = static_cast<T*>(a.out) + c0;
  auto store_out = [&](int j, const P& s) {
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (c0 + j * E + e < a.cols) out[j * E + e] = s.v[e];
  };
  if (ng == 1) {
    for (int j = tid; j < S; j += kThreads) store_out(j, red[j]);
  } else {
    for (int j = tid; j < S; j += kThreads) st_sc1(&slab[size_t(q) * S + j], red[j]);
    unsigned idx = unsigned(q), count = unsigned(ng), stride = 1;
    int lvl_off = 0, lvl_cap = kLsqWideMaxGroups / int(F);
    for (;;) {
      drain_vm();
      __syncthreads();
      const unsigned first = (idx / F) * F;
      const unsigned gsize = count - first < F ? count - first : F;
      if (tid == 0) {
        unsigned* c = &ctr[lvl_off + int(idx / F)];
        const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_ticket = old + 1 == gsize;
        if (s_ticket) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (!s_ticket) return;  // an earlier arriver of the group: the last one carries it
      const unsigned next = (count + F - 1) / F;
      const P* src = slab + size_t(first) * stride * S;
      for (int j = tid; j < S; j += kThreads) {
        P s = ld_sc1(&src[j]);
        for (unsigned m = 1; m < gsize; ++m) {
          const P t = ld_sc1(&src[size_t(m) * stride * S + j]);
#pragma unroll
          for (int e = 0; e < E; ++e) s.v[e] += t.v[e];
        }
        if (next == 1) store_out(j, s);
        else st_sc1(&slab[size_t(first) * stride * S + j], s);
      }
      if (next == 1) break;
      idx /= F;
      count = next;
      stride *= F;
      lvl_off += lvl_cap;
      lvl_cap = (lvl_cap + int(F) - 1) / int(F);
    }
  }
  // this slice of g is written: the task's last slice publishes completion
  drain_vm();
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    uint32_t* done = a.wctr + nslice * kLsqWideCtrPerSlice;
    const unsigned old = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == unsigned(nslice)) {
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      publish_done(a.flag, a.seq);
      publish_peer(a.flag2, a.seq);
    }
  }
}

}  // namespace

hipError_t launch_lsqw(int dtype, const LsqBatch& a, hipStream_t s) {
  const int grid1 = a.block0[a.ntasks];
  int grid2 = 0;
  for (int k = 0; k < a.ntasks; ++k) {
    const LsqTask& t = a.t[k];
    if (t.cols <= kLsqWideSlice || t.cols > kLsqWideMaxCols || t.grid2 < 1 || t.grid2 > kLsqWideMaxGroups || !t.r ||
        !t.wctr)
      return hipErrorInvalidValue;
    grid2 += (t.cols + kLsqWideSlice - 1) / kLsqWideSlice * t.grid2;
  }
  if (grid1 <= 0) return hipErrorInvalidValue;
  if (dtype == MPA_F32) {
    if (batch_armed(a)) hipLaunchKernelGGL((lsqw_resid_kernel<float, true>), dim3(grid1), dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((lsqw_resid_kernel<float, false>), dim3(grid1), dim3(kThreads), 0, s, a);
    hipLaunchKernelGGL((lsqw_grad_kernel<float, 8, 2>), dim3(grid2), dim3(kThreads), 0, s, a);
  } else if (dtype == MPA_F64) {
    if (batch_armed(a)) hipLaunchKernelGGL((lsqw_resid_kernel<double, true>), dim3(grid1), dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((lsqw_resid_kernel<double, false>), dim3(grid1), dim3(kThreads), 0, s, a);
    hipLaunchKernelGGL((lsqw_grad_kernel<double, 16, 1>), dim3(grid2), dim3(kThreads), 0, s, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace mpa
