// Single-pass batched least squares by ITERATE quarters (BASELINE configs[4], "c5"):
//     G_i = A_i^T (A_i X - B_i)      A_i rows x cols bf16, X cols x 64 bf16, B_i rows x 64 bf16
// The fp32 G (cols x 64) does not fit one CU at cols 2048 (512 KiB), but a quarter of its
// iterates does: workgroup q of a QUAD computes, for the quad's rows,
//     R_q = A X[:, 16q .. 16q+15] - B[:, 16q ..]     (16 rows x 16 iterates per block)
//     G[:, 16q .. 16q+15] += A^T R_q                  (cols x 16 fp32 = 128 KiB, registers)
// reading whole rows of A.  The four members of a quad need NO data from each other (each
// owns its iterates), so there is no exchange and no waiting; they read the same rows of A,
// and they are placed to share an XCD (blocks b, b+8, b+16, b+24 of every 32 share one
// under the dispatcher's round-robin, MI355X_MICROARCH.md §Workgroup dispatch), so three of
// the four reads of a block hit that XCD's L2 and HBM sees A about once.  Placement decides
// only speed, never results.
//
// Workgroup = 16 waves (4 per SIMD, <= 128 VGPRs each); wave w owns columns
// [128w, 128w + 128):
//   phase 1  r_w = A[16 rows][its 128 cols] X[its 128 cols][16 iterates]: 4 MFMAs from A
//            fragments loaded straight into registers, two blocks ahead; the 16 partials
//            are summed in LDS in wave order and B subtracted: the residual, split bf16
//            hi + lo;
//   phase 2  G^T[16 iterates][its 256 cols] += res^T A: the wave's A fragments are also
//            written to its own LDS window and read back transposed (ds_read_b64_tr_b16),
//            one K = 32 MFMA per 16-column tile (k 0-15 hi residual, 16-31 lo residual).
// Measured (8 workers x 1 GiB, tools/gpu_lsqq.sh, profiles/r01_lsqq.txt): 3.9-4.1 ms per
// batch against 3.3 ms for the two passes.  HBM fetch is 1.04 x the algorithmic bytes and
// the L2 hit rate 75 % (the quad's sharing works), but the A loads ALONE (every compute
// step, barrier and LDS write switched off, MPA_LSQQ_DBG=31) take 4.0 ms: the four-fold
// L2 -> CU traffic of this layout is delivered at ~8 TB/s chip-wide, so the layout, not
// the arithmetic or the synchronisation, is the bound.
//
// Per-quad-member partial G in a slab, summed over the row groups in group order by the
// member's last arriver (self-resetting counters), the task's last member publishes.
//
// MFMA 16x16x32 bf16 maps (cdna_hip_programming.md §3): A[m=i][k=8g+j], B[k=8g+j][n=i],
// C/D[m=4g+r][n=i]; lane l: i = l & 15, g = l >> 4.
#include <hip/hip_runtime.h>

#include "device_common.hpp"
#include "kernels.hpp"
#include "mpiasyncpools.h"

namespace mpa {
namespace {

using namespace dev;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int K = kLsqbIterates;  // 64
constexpr int Q_NW = 16;            // waves
constexpr int Q_THREADS = 64 * Q_NW;
constexpr int Q_CW = 128;           // columns per wave
constexpr int Q_KS = Q_CW / 32;     // phase-1 k-steps per wave
constexpr int Q_CT = Q_CW / 16;     // phase-2 column tiles per wave
constexpr int Q_AS = Q_CW * 2 + 16;  // LDS bytes per row of a wave's A window (padded)
constexpr int Q_RS = 80;            // residual image: per iterate hi rows 0-15, lo rows 0-15, pad
constexpr int Q_PS = 17;            // partial residual row stride (floats)
constexpr int Q_UNIT = Q_CT * 64;   // f32x4 per wave partial of G (tiles x 64 lanes)

__device__ __forceinline__ f32x4 mfma32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return uint16_t((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_f32(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

__global__ void __launch_bounds__(Q_THREADS) lsqq_kernel(LsqqBatch batch) {
  __shared__ __attribute__((aligned(16))) uint8_t awin[Q_NW][16 * Q_AS];  // per wave: 16 rows x its columns
  __shared__ float part[Q_NW][16 * Q_PS];                                 // per wave partial residual
  __shared__ __attribute__((aligned(16))) uint8_t resimg[16 * Q_RS];
  __shared__ unsigned s_last;

  if (batch.ntasks > 0 && disarmed(batch.t[0].go, batch.t[0].seq)) return;
  const int tid = threadIdx.x, lane = tid & 63, i = lane & 15, g = lane >> 4;
  const int dbg = batch.dbg;  // MPA_LSQQ_DBG timing probes (G wrong): 1 no phase 2, 2 no phase-1
                              // MFMAs, 4 no residual, 8 no barriers, 16 no
                              // window writes, 32 no A loads
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // quad member q and global group: same-XCD quads when the grid is a multiple of 32
  const int b = int(blockIdx.x);
  int q, G_all;
  if ((gridDim.x & 31) == 0) {
    q = (b >> 3) & 3;
    G_all = (b >> 5) * 8 + (b & 7);
  } else {
    q = b & 3;
    G_all = b >> 2;
  }
  if (G_all >= batch.grp0[batch.ntasks]) return;
  int ti = 0;
  while (ti + 1 < batch.ntasks && G_all >= batch.grp0[ti + 1]) ++ti;
  const LsqqTask& a = batch.t[ti];
  const int grp = G_all - batch.grp0[ti];
  const int ngroups = batch.grp0[ti + 1] - batch.grp0[ti];
  const int64_t rows = a.rows;
  const int cols = a.cols;
  const int nw = (cols + Q_CW - 1) / Q_CW;  // waves with columns
  const int64_t nblocks = (rows + 15) / 16;
  const int nb = nblocks > grp ? int((nblocks - grp + ngroups - 1) / ngroups) : 0;  // this group's blocks
  const int c0 = Q_CW * wave;
  const int nks = cols > c0 ? ((cols - c0) < Q_CW ? (cols - c0) : Q_CW) / 32 : 0;  // this wave's k-steps
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(a.A);
  const uint16_t* __restrict__ Bm = static_cast<const uint16_t*>(a.B);
  const uint16_t* __restrict__ X = static_cast<const uint16_t*>(a.X);

  // phase-1 B operands X[c0 + 32 s + 8 g + j][16 q + i]; k-steps past cols are zero
  bf16x8 XF[Q_KS];
#pragma unroll
  for (int s = 0; s < Q_KS; ++s) {
    s16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + 32 * s + 8 * g + j;
      v[j] = s < nks ? short(X[size_t(c) * K + 16 * q + i]) : short(0);
    }
    XF[s] = __builtin_bit_cast(bf16x8, v);
  }
  f32x4 acc[Q_CT];  // G^T[16 q + 4 g + r][c0 + 16 ct + i]
#pragma unroll
  for (int ct = 0; ct < Q_CT; ++ct) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A and B through buffer loads: one 32-bit offset per lane, the block's base and extent
  // in scalar registers, and the hardware range check returns 0 for rows past the end and
  // for k-steps past the columns (soffset pushed out of range), so no load is clamped or
  // predicated (a load under a branch made the compiler drain every load in flight before
  // the MFMAs, lsqb_kernel.hip pass 1) and no 64-bit address is held per load
  typedef bf16x8 Frags[Q_KS];
  const int last = nb > 0 ? nb - 1 : 0;
  auto blockrow = [&](int t) -> int64_t { return (int64_t(grp) + int64_t(t < last ? t : last) * ngroups) * 16; };
  auto rsrc = [&](const uint16_t* base, int64_t row0, int64_t row_elems) {
    const int64_t left = (rows - row0) * row_elems * 2;
    const int nrec = left > 0x7FFFFFF0 ? 0x7FFFFFF0 : int(left);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(base + row0 * row_elems), 0, nrec, 0x00020000);
  };
  const int a_off = int((int64_t(i) * a.lda + c0 + 8 * g) * 2);
  auto load_a = [&](Frags& F, int t) {
    if (dbg & 32) {  // probe: no A loads
#pragma unroll
      for (int s = 0; s < Q_KS; ++s) F[s] = XF[s];
      return;
    }
    const auto rs = rsrc(A, blockrow(t), a.lda);
#pragma unroll
    for (int s = 0; s < Q_KS; ++s)
      F[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, a_off, s < nks ? 64 * s : 0x40000000, 0));
  };
  // the reduction thread's B value (row tid >> 4, iterate 16 q + (tid & 15)), threads < 256
  const int rrow = (tid >> 4) & 15, rit = tid & 15;
  const int b_off = (rrow * K + 16 * q + rit) * 2;
  auto load_b = [&](int t) -> uint16_t {
    return __builtin_amdgcn_raw_buffer_load_b16(rsrc(Bm, blockrow(t), K), b_off, 0, 0);
  };

  const int q4 = (lane >> 2) & 3, p4 = lane & 3;
  uint8_t* win = awin[wave];
  auto step = [&](int t, Frags& F, Frags& N, uint16_t& Bc, uint16_t& Bn) {
    load_a(N, t + 2);
    Bn = load_b(t + 2);
    // phase 1: this wave's partial residual, and its A fragments into its window
    f32x4 r1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < Q_KS && !(dbg & 2); ++s) r1 = mfma32(F[s], XF[s], r1);
#pragma unroll
    for (int s = 0; s < Q_KS && !(dbg & 16); ++s) *reinterpret_cast<bf16x8*>(win + i * Q_AS + 64 * s + 16 * g) = F[s];
#pragma unroll
    for (int r = 0; r < 4; ++r) part[wave][(4 * g + r) * Q_PS + i] = r1[r];
    if (!(dbg & 8)) __syncthreads();
    // residual = partials in wave order - B, split hi + lo (threads 0-255: row, iterate)
    if (tid < 256 && !(dbg & 4)) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < Q_NW; ++w) v += part[w][rrow * Q_PS + rit];
      const int64_t row = blockrow(t) + rrow;
      const float x = row < rows ? v - bf16_f32(Bc) : 0.f;
      const uint16_t hv = bf16_rne(x), lv = bf16_rne(x - bf16_f32(hv));
      *reinterpret_cast<uint16_t*>(resimg + rit * Q_RS + 2 * rrow) = hv;
      *reinterpret_cast<uint16_t*>(resimg + rit * Q_RS + 32 + 2 * rrow) = lv;
    }
    if (!(dbg & 8)) __syncthreads();
    // phase 2: G^T[16 iterates][c0 + 16 ct + i] += res^T A (K = 16 rows hi + 16 rows lo)
    const bf16x8 ra = *reinterpret_cast<const bf16x8*>(resimg + i * Q_RS + 16 * g);
    const uint8_t* sb = win + (8 * (g & 1) + q4) * Q_AS + 8 * p4;
#pragma unroll
    for (int ct = 0; ct < Q_CT && !(dbg & 1); ++ct) {
      const s16x4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sb + 32 * ct));
      const s16x4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sb + 4 * Q_AS + 32 * ct));
      const bf16x8 bt = __builtin_bit_cast(bf16x8, __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7));
      acc[ct] = mfma32(ra, bt, acc[ct]);
      // transposed reads four tiles ahead at most: hoisting all 32 cost 64 VGPRs
      if ((ct & 1) == 1) __builtin_amdgcn_sched_barrier(0);
    }
  };

  if (nb > 0) {
    Frags FA, FB, FC;
    uint16_t BA, BB, BC;
    load_a(FA, 0);
    BA = load_b(0);
    load_a(FB, 1);
    BB = load_b(1);
    int t = 0;
    for (;;) {
      step(t, FA, FC, BA, BC);
      if (++t >= nb) break;
      step(t, FB, FA, BB, BA);
      if (++t >= nb) break;
      step(t, FC, FB, BC, BB);
      if (++t >= nb) break;
    }
  }

  // this wave's G partial -> slab[grp][q][wave][ct][lane] (waves past the columns skip)
  float* slab = static_cast<float*>(a.slab);
  const size_t unit = size_t(nw) * Q_UNIT;  // f32x4 per (group, member)
  if (wave < nw) {
    f32x4* part_g = reinterpret_cast<f32x4*>(slab) + (size_t(grp) * 4 + q) * unit + size_t(wave) * Q_UNIT;
#pragma unroll
    for (int ct = 0; ct < Q_CT; ++ct) part_g[ct * 64 + lane] = acc[ct];
  }
  drain_vm();
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == unsigned(ngroups - 1);
    if (s_last) {
      // every group of this member has arrived: reset for the next launch (stream-ordered)
      __hip_atomic_store(&a.ctr[q], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      drain_vm();
    }
  }
  __syncthreads();
  if (!s_last) return;
  // member q's last arriver: sum the groups in group order, write G[col][16 q + ..]
  const f32x4* base = reinterpret_cast<const f32x4*>(slab) + size_t(q) * unit;
  const size_t gstride = 4 * unit;
  float* out = static_cast<float*>(a.out);
  for (int j = tid; j < int(unit); j += Q_THREADS) {
    f32x4 s0 = base[j];
    for (int gq = 1; gq < ngroups; ++gq) s0 += base[size_t(gq) * gstride + j];
    // j = (w * Q_CT + ct) * 64 + l -> column Q_CW w + 16 ct + (l & 15), iterates 16 q + 4 (l >> 4) + r
    const int l = j & 63, ct = (j >> 6) % Q_CT, w = (j >> 6) / Q_CT;
    const int col = Q_CW * w + 16 * ct + (l & 15);
    if (col < cols) *reinterpret_cast<f32x4*>(out + size_t(col) * K + 16 * q + 4 * (l >> 4)) = s0;
  }
  drain_vm();
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[4], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == 3u) {
      __hip_atomic_store(&a.ctr[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      publish_done(a.flag, a.seq);
    }
  }
}

}  // namespace

hipError_t launch_lsqq(const LsqqBatch& a, hipStream_t s) {
  const int groups = a.grp0[a.ntasks];
  if (groups <= 0 || a.ntasks < 1 || a.ntasks > kMaxLsqTasks) return hipErrorInvalidValue;
  for (int k = 0; k < a.ntasks; ++k)
    if (a.t[k].cols <= 0 || a.t[k].cols > Q_NW * Q_CW || a.t[k].cols % 32) return hipErrorInvalidValue;
  hipLaunchKernelGGL(lsqq_kernel, dim3(4 * groups), dim3(Q_THREADS), 0, s, a);
  return hipGetLastError();
}

}  // namespace mpa
