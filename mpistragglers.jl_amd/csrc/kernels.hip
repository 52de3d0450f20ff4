// gfx950 (CDNA4) kernels of the asyncmap! hot path.
//
//   lsq_grad_kernel   worker compute g = A^T (A x - b): ONE pass over A (the BASELINE
//                     workload in the reference's compute slot, examples/iterative_example.jl:74)
//   exchange_kernel   the reference's byte copies `isendbufs[i] .= sendbuf` (:130,:178) and
//                     `recvbufs[i] .= irecvbufs[i]` (:108,:167,:216), batched per flush
//   kmap_task_kernel  the reference's test worker programs (test/kmap1.jl, test/kmap2.jl)
//   delay_kernel      straggler emulation (the reference's `sleep(rand())`, iterative_example.jl:74)
//   aggregate_kernel  coordinator consumption of fresh chunks (iterative_example.jl:41-46)
//   generate_kernel   Philox4x32-10 synthetic data, bit-identical to oracle/philox.h
//
// Completion protocol (every worker task kernel): the reply chunk is stored, released at
// agent scope, and the LAST writer publishes `seq` into the worker's host-pinned flag with
// a system-scope release; the coordinator thread polls that word (MPI.Test!/Waitany!).
#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "mpiasyncpools.h"

namespace mpa {

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

template <typename T>
struct alignas(16) Pack {
  static constexpr int E = 16 / sizeof(T);
  T v[E];
};

__device__ __forceinline__ unsigned long long rt_now() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// One lane publishes completion of a task whose stores every wave of this workgroup has
// drained (caller: drain_vm() + __syncthreads() first).
__device__ __forceinline__ void publish_done(const Publish& p) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  drain_vm();
  __threadfence_system();
  drain_vm();
  __hip_atomic_store(p.flag, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void report_error(const Publish& p, unsigned code) {
  __hip_atomic_fetch_or(p.err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------------------
// lsq_grad_kernel<T, VPL, RB>
//
// Layout: A is row-major (rows x lda, lda % E == 0).  A wave owns whole rows: lane l holds
// the 16-B vectors v*64 + l (v < VPL) of a row, so every load instruction of the wave reads
// 1 KiB contiguous.  x and the running g live in registers for the whole kernel.  Per row:
//   dot = wave_sum(sum_v a_v . x_v);  r = dot - b[row];  g_v += r * a_v
// i.e. A is read from HBM exactly once (the single-pass requirement of SURVEY.md §7).
// Rows are dealt to waves in tiles of RB rows, grid-strided so the whole grid sweeps one
// contiguous region of A at a time.
//
// Cross-workgroup reduction (deterministic, no float atomics): the 4 waves of a workgroup
// add their g in LDS in wave order, the workgroup stores its partial into slab[block][:],
// then takes a ticket on a monotonic arrival counter.  The last R arrivers (R = 4*VPL)
// each wait for the counter to reach the grid size, then sum one 256-B column block of
// the slab over all workgroups in block order, and store it into the reply chunk.  The
// last of the R reducers publishes completion.  Spins are bounded (pub.spin_ticks).
// ---------------------------------------------------------------------------------------
template <typename T, int VPL, int RB>
__global__ void __launch_bounds__(kThreads) lsq_grad_kernel(LsqBatch batch) {
  using P = Pack<T>;
  constexpr int E = P::E;
  constexpr int R = 4 * VPL;            // reducers; each owns 16 vectors = 256 B of columns
  __shared__ P red[VPL * 64];           // workgroup partial (VPL*64*E columns)
  __shared__ P part[16][16];            // reducer phase partials
  __shared__ unsigned s_ticket;

  // which task of the batch this workgroup serves (wave-uniform scan over <= 16 entries)
  int ti = 0;
  while (ti + 1 < batch.ntasks && int(blockIdx.x) >= batch.block0[ti + 1]) ++ti;
  const LsqTask& a = batch.t[ti];
  const int blk = int(blockIdx.x) - batch.block0[ti];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const T* __restrict__ A = static_cast<const T*>(a.A);
  const T* __restrict__ bv = static_cast<const T*>(a.b);
  const T* __restrict__ xv = static_cast<const T*>(a.x);

  // x slice and column mask (columns >= cols contribute nothing)
  P xr[VPL], g[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c0 = (v * 64 + lane) * E;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      xr[v].v[e] = (c0 + e < a.cols) ? xv[c0 + e] : T(0);
      g[v].v[e] = T(0);
    }
  }
  bool vok[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) vok[v] = (v * 64 + lane) * E < a.cols;

  const int64_t rows = a.rows;
  const int64_t step = int64_t(a.grid) * kWaves * RB;
  for (int64_t base = (int64_t(blk) * kWaves + wave) * RB; base < rows; base += step) {
    P d[RB][VPL];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int64_t r = base + rb;
      const P* row = reinterpret_cast<const P*>(A + r * a.lda);
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        if (r < rows && vok[v]) {
          d[rb][v] = row[v * 64 + lane];
        } else {
#pragma unroll
          for (int e = 0; e < E; ++e) d[rb][v].v[e] = T(0);
        }
      }
    }
    T dot[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      T s = T(0);
#pragma unroll
      for (int v = 0; v < VPL; ++v)
#pragma unroll
        for (int e = 0; e < E; ++e) s += d[rb][v].v[e] * xr[v].v[e];
      dot[rb] = s;
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) dot[rb] = wave_sum(dot[rb]);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int64_t r = base + rb;
      const T res = (r < rows) ? dot[rb] - bv[r] : T(0);
#pragma unroll
      for (int v = 0; v < VPL; ++v)
#pragma unroll
        for (int e = 0; e < E; ++e) g[v].v[e] += res * d[rb][v].v[e];
    }
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
  P* slab = static_cast<P*>(a.slab) + size_t(blk) * (VPL * 64);
  for (int j = tid; j < VPL * 64; j += kThreads) slab[j] = red[j];
  drain_vm();
  __syncthreads();

  const unsigned G = unsigned(a.grid);
  const unsigned base0 = unsigned((a.seq - 1ull) * G);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_ticket = old - base0;
  }
  __syncthreads();
  const unsigned ticket = s_ticket;
  if (ticket + R < G) return;  // not one of the last R arrivers
  const int k = int(ticket + R - G);  // reducer index 0..R-1

  if (tid == 0) {
    const unsigned long long t0 = rt_now();
    while (__hip_atomic_load(&a.ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - base0 < G) {
      __builtin_amdgcn_s_sleep(2);
      if (rt_now() - t0 > batch.spin_ticks) {
        __hip_atomic_fetch_or(batch.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    drain_vm();
  }
  __syncthreads();

  // column block k: vectors [16k, 16k+16) of every slab row, summed over blocks in order
  const int vv = tid & 15, ph = tid >> 4;
  const P* src = static_cast<const P*>(a.slab) + k * 16 + vv;
  P acc;
#pragma unroll
  for (int e = 0; e < E; ++e) acc.v[e] = T(0);
  for (unsigned b = unsigned(ph); b < G; b += 16) {
    const P t = src[size_t(b) * (VPL * 64)];
#pragma unroll
    for (int e = 0; e < E; ++e) acc.v[e] += t.v[e];
  }
  part[ph][vv] = acc;
  __syncthreads();
  if (ph == 0) {
    P s = part[0][vv];
#pragma unroll
    for (int q = 1; q < 16; ++q)
#pragma unroll
      for (int e = 0; e < E; ++e) s.v[e] += part[q][vv].v[e];
    T* out = static_cast<T*>(a.out);
    const int c0 = (k * 16 + vv) * E;
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (c0 + e < a.cols) out[c0 + e] = s.v[e];
  }
  drain_vm();
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned base1 = unsigned((a.seq - 1ull) * unsigned(R));
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old - base1 == unsigned(R - 1)) {
      Publish p{a.flag, batch.err, a.seq, 0};
      publish_done(p);
    }
  }
}

// ---------------------------------------------------------------------------------------
__device__ void block_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {
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
  const int npb = a.npost * a.bpp;
  if (b < npb) {
    const int item = b / a.bpp, part = b % a.bpp;
    const uint64_t off = uint64_t(part) * a.ppart;
    if (off >= a.sl) return;
    const uint64_t len = (a.sl - off) < a.ppart ? (a.sl - off) : a.ppart;
    block_copy(a.isendbuf + uint64_t(a.post[item]) * a.sl + off, a.sendbuf + off, len);
  } else {
    const int hb = b - npb;
    const int item = hb / a.bph, part = hb % a.bph;
    const uint64_t off = uint64_t(part) * a.hpart;
    if (off >= a.rl) return;
    const uint64_t len = (a.rl - off) < a.hpart ? (a.rl - off) : a.hpart;
    const uint64_t c = uint64_t(a.harv[item]) * a.rl + off;
    block_copy(a.recvbuf + c, a.irecvbuf + c, len);
  }
}

// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) kmap_task_kernel(KmapArgs a) {
  if (a.kind == MPA_TASK_ECHO) {
    const uint64_t m = a.sl < a.rl ? a.sl : a.rl;
    for (uint64_t j = threadIdx.x; j < a.rl; j += blockDim.x) a.out[j] = j < m ? a.x[j] : uint8_t(0);
  } else if (threadIdx.x == 0) {
    double v[3] = {a.rank, double(a.pub.seq), 0.0};  // t == tasks served (kmap2.jl:116-118)
    uint8_t* vb = reinterpret_cast<uint8_t*>(v);
    if (a.kind == MPA_TASK_KMAP2) {
      for (uint64_t j = 0; j < 8 && j < a.sl; ++j) vb[16 + j] = a.x[j];  // epoch = recvbuf[1]
    }
    const uint64_t m = a.kind == MPA_TASK_KMAP1 ? 8 : 24;
    for (uint64_t j = 0; j < a.rl; ++j) a.out[j] = j < m ? vb[j] : uint8_t(0);
  }
  drain_vm();
  __syncthreads();
  if (threadIdx.x == 0) publish_done(a.pub);
}

__global__ void delay_kernel(unsigned long long ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = rt_now();
  while (rt_now() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}

// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(kThreads) aggregate_kernel(AggregateArgs a) {
  const T* c = static_cast<const T*>(a.chunks);
  T* out = static_cast<T*>(a.out);
  for (int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < a.elems;
       j += int64_t(gridDim.x) * blockDim.x) {
    double s = 0.0;
    for (int64_t i = 0; i < a.n; ++i)
      if (a.w[i] != 0.0) s += a.w[i] * double(c[i * a.stride + j]);
    out[j] = a.update ? T(double(out[j]) - a.eta * s) : T(s);
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

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return uint16_t((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
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

template <typename T, int VPL, int RB>
hipError_t lsq_go(const LsqBatch& a, hipStream_t s) {
  const int grid = a.block0[a.ntasks];
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL((lsq_grad_kernel<T, VPL, RB>), dim3(grid), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

template <typename T>
constexpr int vpl_for(int cols) {
  constexpr int per = 64 * Pack<T>::E;
  return (cols + per - 1) / per;
}

}  // namespace

// variant table: (VPL, RB) per dtype
int lsq_cols_pad(int dtype, int cols) {
  if (cols <= 0) return 0;
  if (dtype == MPA_F32) {
    const int v = vpl_for<float>(cols);
    const int vp = v <= 1 ? 1 : v <= 2 ? 2 : v <= 4 ? 4 : v <= 8 ? 8 : 0;
    return vp * 64 * 4;
  }
  if (dtype == MPA_F64) {
    const int v = vpl_for<double>(cols);
    const int vp = v <= 1 ? 1 : v <= 2 ? 2 : v <= 4 ? 4 : v <= 8 ? 8 : v <= 16 ? 16 : 0;
    return vp * 64 * 2;
  }
  return 0;
}

int lsq_reducers(int dtype, int cols) {
  const int cp = lsq_cols_pad(dtype, cols);
  return cp ? 4 * (cp / (64 * (dtype == MPA_F64 ? 2 : 4))) : 0;
}

int lsq_rows_per_wave_iter(int dtype, int cols) {
  const int cp = lsq_cols_pad(dtype, cols);
  if (dtype == MPA_F32) return cp <= 1024 ? 4 : 2;
  return cp <= 256 ? 4 : cp <= 1024 ? 2 : 1;
}

hipError_t launch_lsq(int dtype, int cols, const LsqBatch& a, hipStream_t s) {
  const int cp = lsq_cols_pad(dtype, cols);
  if (dtype == MPA_F32) {
    switch (cp) {
      case 256: return lsq_go<float, 1, 4>(a, s);
      case 512: return lsq_go<float, 2, 4>(a, s);
      case 1024: return lsq_go<float, 4, 4>(a, s);
      case 2048: return lsq_go<float, 8, 2>(a, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (dtype == MPA_F64) {
    switch (cp) {
      case 128: return lsq_go<double, 1, 4>(a, s);
      case 256: return lsq_go<double, 2, 4>(a, s);
      case 512: return lsq_go<double, 4, 2>(a, s);
      case 1024: return lsq_go<double, 8, 2>(a, s);
      case 2048: return lsq_go<double, 16, 1>(a, s);
      default: return hipErrorInvalidValue;
    }
  }
  return hipErrorInvalidValue;
}

hipError_t launch_exchange(const ExchangeArgs& a, hipStream_t s) {
  const int grid = a.npost * a.bpp + a.nharv * a.bph;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(exchange_kernel, dim3(grid), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_kmap(const KmapArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(kmap_task_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_delay(unsigned long long ticks, hipStream_t s) {
  hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, s, ticks);
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

hipError_t launch_generate(void* out, int dtype, uint64_t seed, uint32_t stream, uint64_t e0, int64_t count,
                           double scale, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  const uint64_t quads = ((e0 + uint64_t(count) + 3) >> 2) - (e0 >> 2);
  const uint64_t want = (quads + kThreads - 1) / kThreads;
  const int grid = int(want < 8192 ? want : 8192);
  hipLaunchKernelGGL(generate_kernel, dim3(grid), dim3(kThreads), 0, s, out, dtype, seed, stream, e0, count, scale);
  return hipGetLastError();
}

}  // namespace mpa
