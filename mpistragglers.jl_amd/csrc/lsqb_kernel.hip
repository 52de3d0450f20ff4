// The batched multi-iterate worker compute (BASELINE configs[4], "c5"):
//     G_i = A_i^T (A_i X - B_i)       A_i rows x cols bf16, X cols x 64 bf16 (the message),
//                                     B_i rows x 64 bf16, G_i cols x 64 fp32 (the reply)
// placed in the reference's compute slot (examples/iterative_example.jl:74 sleeps there).
// Unlike the one-iterate kernel (lsq_kernel.hip) this is a real contraction, so both
// products run on the bf16 MFMA (v_mfma_f32_16x16x32_bf16, fp32 accumulate).
//
// Why two passes.  The fp32 accumulator of G_i is cols x 64 x 4 B = 512 KiB at cols 2048:
// the whole register file of a CU, so no workgroup can hold G for all columns while it
// streams full rows of A (which the residual needs).  The task therefore runs as
//   pass 1  lsqb_resid_kernel: R = A X - B, one HBM pass over A, R stored split into
//           bf16 hi + lo (R = hi + lo to ~2^-17 relative) in the k-packed layout pass 2's
//           MFMA operand wants (8 consecutive rows of one iterate = 16 contiguous bytes);
//   pass 2  lsqb_grad_kernel: G = A^T (R_hi + R_lo), a second HBM pass over A, workgroups
//           = (row range, 256-column slice); A tiles are staged in LDS and read back
//           TRANSPOSED by ds_read_b64_tr_b16 (the MFMA's K = rows); the row-range partials
//           of a slice are summed in fixed order by the slice's last arriver (no float
//           atomics, bitwise reproducible for a given grid) and the task's last slice
//           publishes completion.
// DESIGN.md §Kernels states the two-pass roofline (A read twice) and the single-pass plan.
//
// MFMA fragment maps (16x16x32 bf16, cdna_hip_programming.md §3): lane l, g = l>>4, i = l&15:
//   A operand  A[m = i][k = 8g + j]   B operand  B[k = 8g + j][n = i]   (j = 0..7)
//   C/D        D[m = 4g + r][n = i]   (r = 0..3)
#include <hip/hip_runtime.h>

#include "device_common.hpp"
#include "kernels.hpp"
#include "mpiasyncpools.h"

namespace mpa {
namespace {

using namespace dev;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int K = kLsqbIterates;  // 64 iterates = 4 MFMA tiles of 16

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ uint4 ld16(const void* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ uint4 ld16_nt(const void* p) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// B operand of one 16x16x32 MFMA from a row-major LDS tile by two hardware transposed
// reads: rows k0+8g+q (element q) and k0+8g+4+q (element 4+q), columns n0..n0+15 (lane i
// gets column n0+i).  Lane 4q+p of each 16-lane group addresses row q, columns 4p..4p+3.
__device__ __forceinline__ bf16x8 tr_operand(const uint8_t* tile, int stride, int k0, int n0_bytes, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const uint8_t* a0 = tile + (k0 + 8 * g + q) * stride + n0_bytes + 8 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * stride));
  const s16x4 v0 = lo, v1 = hi;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 w = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, w);
}

__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return uint16_t((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

__device__ __forceinline__ int task_of(const int* block0, int ntasks) {
  int ti = 0;
  while (ti + 1 < ntasks && int(blockIdx.x) >= block0[ti + 1]) ++ti;
  return ti;
}

// ---------------------------------------------------------------------------------------
// pass 1: R = A X - B.  Workgroup = 4 waves x 64 rows; X streams through LDS in chunks of
// 128 rows (double buffered, shared by the 4 waves), A goes straight to registers as the
// MFMA A operand (each lane 16 B; the four lanes of a row read 64 contiguous bytes).
constexpr int P1_KC = 128;          // X rows per LDS chunk
constexpr int P1_XS = K * 2 + 16;   // LDS bytes per X row (pad: 2-way tr reads at most)
constexpr int P1_WG_ROWS = 256;

__global__ void __launch_bounds__(kThreads) lsqb_resid_kernel(LsqbBatch batch) {
  __shared__ __attribute__((aligned(16))) uint8_t xs[2][P1_KC * P1_XS];
  const int ti = task_of(batch.block1, batch.ntasks);
  const LsqbTask& a = batch.t[ti];
  const int blk = int(blockIdx.x) - batch.block1[ti];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t rows = a.rows;
  const int cols = a.cols;
  const int nblocks = int((rows + P1_WG_ROWS - 1) / P1_WG_ROWS);
  if (blk >= nblocks) return;  // whole workgroup
  const int nchunk = (cols + P1_KC - 1) / P1_KC;
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(a.A);
  const uint16_t* __restrict__ Bm = static_cast<const uint16_t*>(a.B);
  const uint8_t* __restrict__ X = static_cast<const uint8_t*>(a.X);
  uint8_t* __restrict__ R = static_cast<uint8_t*>(a.R);

  // X chunk c: rows [c*KC, c*KC + KC); thread t moves 16-B piece (t&7) of rows (t>>3) + 32q
  uint4 xr[4];
  auto load_x = [&](int c) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = c * P1_KC + (tid >> 3) + 32 * q;
      xr[q] = r < cols ? ld16(X + size_t(r) * (K * 2) + (tid & 7) * 16) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<uint4*>(&xs[buf][((tid >> 3) + 32 * q) * P1_XS + (tid & 7) * 16]) = xr[q];
  };

  load_x(0);
  store_x(0);
  __syncthreads();
  int cur = 0;
  for (int rb = blk; rb < nblocks; rb += a.grid1) {
    const int64_t row_w = int64_t(rb) * P1_WG_ROWS + wave * 64;
    const uint16_t* arow[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      int64_t r = row_w + 16 * m + i;
      r = r < rows ? r : rows - 1;
      arow[m] = A + r * a.lda + 8 * g;
    }
    f32x4 acc[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int c = 0; c < nchunk; ++c) {
      const bool last_chunk = c + 1 == nchunk;
      const bool more = !(last_chunk && rb + a.grid1 >= nblocks);
      if (more) load_x(last_chunk ? 0 : c + 1);
      const uint8_t* tile = xs[cur];
#pragma unroll
      for (int s = 0; s < P1_KC / 32; ++s) {
        const int k0 = c * P1_KC + 32 * s;
        if (k0 >= cols) break;  // wave-uniform (cols % 32 == 0)
        bf16x8 af[4], bf[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) af[m] = __builtin_bit_cast(bf16x8, ld16_nt(arow[m] + k0));
#pragma unroll
        for (int t = 0; t < 4; ++t) bf[t] = tr_operand(tile, P1_XS, 32 * s, 32 * t, lane);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[m][t] = mfma(af[m], bf[t], acc[m][t]);
      }
      if (more) store_x(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }

    // R = acc - B, split hi/lo, into the k-packed layout: entry (row/8, iterate) = 32 B =
    // hi[8] | lo[8] (element row%8).  This lane holds rows row_w+16m+4g+r, iterate 16t+i.
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t r0 = row_w + 16 * m + 4 * g;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int it = 16 * t + i;
        uint16_t hi[4], lo[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = r0 + r;
          float v = 0.f;
          if (row < rows) v = acc[m][t][r] - bf16_to_f32(Bm[row * K + it]);
          hi[r] = bf16_rne(v);
          lo[r] = bf16_rne(v - bf16_to_f32(hi[r]));
        }
        uint8_t* e = R + ((size_t(r0 >> 3) * K + it) * 32) + (g & 1) * 8;
        *reinterpret_cast<uint2*>(e) = make_uint2(uint32_t(hi[0]) | (uint32_t(hi[1]) << 16),
                                                  uint32_t(hi[2]) | (uint32_t(hi[3]) << 16));
        *reinterpret_cast<uint2*>(e + 16) = make_uint2(uint32_t(lo[0]) | (uint32_t(lo[1]) << 16),
                                                       uint32_t(lo[2]) | (uint32_t(lo[3]) << 16));
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// pass 2: G = A^T R.  Workgroup (range rho, slice sigma): rows [32*s_begin, 32*s_end) x
// columns [256 sigma, 256 sigma + 256); wave w owns columns 64w..64w+63 of the slice and all
// 64 iterates (acc 4 x 4 tiles: G^T[iterate][column]).  Per k-step (32 rows) the A tile
// (32 x 256 bf16 = 16 KiB) is staged in LDS (double buffered, loaded one step ahead) and
// read transposed as the B operand; R_hi / R_lo fragments are one 16-B load each.
constexpr int P2_CW = 256;
constexpr int P2_AS = P2_CW * 2 + 16;
constexpr int P2_PART = K * P2_CW;  // floats per workgroup partial

__global__ void __launch_bounds__(kThreads) lsqb_grad_kernel(LsqbBatch batch) {
  __shared__ __attribute__((aligned(16))) uint8_t as_[2][32 * P2_AS];
  __shared__ unsigned s_last;
  const int ti = task_of(batch.block2, batch.ntasks);
  const LsqbTask& a = batch.t[ti];
  const int blk = int(blockIdx.x) - batch.block2[ti];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nrange = a.nrange, nslice = a.nslice;
  const int rho = blk % nrange, sigma = blk / nrange;  // same rho -> same blk % 8 (XCD)
  const int64_t rows = a.rows;
  const int cols = a.cols;
  const int64_t S = (rows + 31) / 32;
  const int64_t s_begin = S * rho / nrange, s_end = S * (rho + 1) / nrange;
  const int c0 = sigma * P2_CW;
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(a.A);
  const uint8_t* __restrict__ R = static_cast<const uint8_t*>(a.R);

  // tile loader: thread t moves 16 B (8 columns) = chunk (t&31) of rows (t>>5) + 8q
  const int lc = c0 + 8 * (tid & 31);
  const bool lc_ok = lc < cols;
  uint4 tr_[4];
  auto load_tile = [&](int64_t s) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int64_t r = 32 * s + (tid >> 5) + 8 * q;
      r = r < rows ? r : rows - 1;  // rows past the end meet R = 0 (pass 1 zero-fills)
      tr_[q] = lc_ok ? ld16_nt(A + r * a.lda + lc) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<uint4*>(&as_[buf][((tid >> 5) + 8 * q) * P2_AS + 16 * (tid & 31)]) = tr_[q];
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (s_begin < s_end) {
    load_tile(s_begin);
    store_tile(0);
  }
  __syncthreads();
  int cur = 0;
  for (int64_t s = s_begin; s < s_end; ++s) {
    const bool more = s + 1 < s_end;
    if (more) load_tile(s + 1);
    bf16x8 rh[4], rl[4], bf[4];
    const uint8_t* re = R + ((size_t(4 * s + g) * K + i) * 32);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      rh[u] = __builtin_bit_cast(bf16x8, ld16(re + size_t(16 * u) * 32));
      rl[u] = __builtin_bit_cast(bf16x8, ld16(re + size_t(16 * u) * 32 + 16));
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) bf[t] = tr_operand(as_[cur], P2_AS, 0, 2 * (64 * wave + 16 * t), lane);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[u][t] = mfma(rh[u], bf[t], acc[u][t]);
        acc[u][t] = mfma(rl[u], bf[t], acc[u][t]);
      }
    if (more) store_tile(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // partial of this workgroup: slab[(rho * nslice + sigma)][wave][u][t][lane][4]
  float* part = static_cast<float*>(a.slab) + size_t(rho * nslice + sigma) * P2_PART;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t)
      *reinterpret_cast<f32x4*>(part + ((((wave * 4 + u) * 4 + t) * 64 + lane) * 4)) = acc[u][t];
  drain_vm();
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[sigma], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old - a.sbase) == unsigned(nrange - 1);
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      drain_vm();
    }
  }
  __syncthreads();
  if (!s_last) return;

  // the slice's last arriver: sum the nrange partials in range order, write G[col][iterate]
  const f32x4* base = reinterpret_cast<const f32x4*>(static_cast<const float*>(a.slab) + size_t(sigma) * P2_PART);
  const size_t rstride = size_t(nslice) * (P2_PART / 4);
  float* out = static_cast<float*>(a.out);
  for (int j = tid; j < P2_PART / 4; j += kThreads) {
    f32x4 s0 = base[j], s1 = f32x4{0.f, 0.f, 0.f, 0.f};
    int r = 1;
    for (; r + 1 < nrange; r += 2) {
      s0 += base[size_t(r) * rstride + j];
      s1 += base[size_t(r + 1) * rstride + j];
    }
    if (r < nrange) s0 += base[size_t(r) * rstride + j];
    s0 += s1;
    // j = ((w*4 + u)*4 + t)*64 + l  ->  column c0 + 64w + 16t + (l&15), iterates 16u + 4(l>>4) + r
    const int l = j & 63, t = (j >> 6) & 3, u = (j >> 8) & 3, w = j >> 10;
    const int col = c0 + 64 * w + 16 * t + (l & 15);
    if (col < cols) {
      float* o = out + size_t(col) * K + 16 * u + 4 * (l >> 4);
      *reinterpret_cast<f32x4*>(o) = s0;
    }
  }
  drain_vm();
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[kLsqbMaxSlices], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old - a.tbase == unsigned(nslice - 1)) publish_done(a.flag, a.seq);
  }
}

}  // namespace

hipError_t launch_lsqb(const LsqbBatch& a, hipStream_t s) {
  const int g1 = a.block1[a.ntasks], g2 = a.block2[a.ntasks];
  if (g1 <= 0 || g2 <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(lsqb_resid_kernel, dim3(g1), dim3(kThreads), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(lsqb_grad_kernel, dim3(g2), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace mpa
