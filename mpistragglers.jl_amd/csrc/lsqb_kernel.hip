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
// pass 1: R = A X - B.  Workgroup = 8 waves x 32 rows (2 MFMA row tiles per wave); X
// streams through LDS in chunks of 128 rows (double buffered, shared by the 8 waves); A
// goes straight to registers as the MFMA A operand (each lane 16 B; the four lanes of a
// row read 64 contiguous bytes), prefetched one whole chunk (4 k-steps, 8 KiB per wave)
// ahead so every CU keeps >= 64 KiB of HBM reads in flight (MI355X_MICROARCH.md §HBM).
constexpr int P1_THREADS = 512;
constexpr int P1_KC = 128;          // X rows per LDS chunk = 4 k-steps of 32
constexpr int P1_XS = K * 2 + 16;   // LDS bytes per X row (pad: 2-way tr reads at most)
constexpr int P1_WG_ROWS = 256;     // 8 waves x 32 rows

template <bool ARMED>
__global__ void __launch_bounds__(P1_THREADS) lsqb_resid_chunked_kernel(LsqbBatch batch) {
  __shared__ __attribute__((aligned(16))) uint8_t xs[2][P1_KC * P1_XS];
  const int ti = task_of(batch.block1, batch.ntasks);
  const LsqbTask& a = batch.t[ti];
  const int blk = int(blockIdx.x) - batch.block1[ti];
  if constexpr (ARMED)  // device-armed (pass 2 follows on the stream)
    if (!wait_door(a.door, a.seq, batch.spin_ticks, batch.err)) return;
  if (disarmed(a.go, a.seq)) return;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t rows = a.rows;
  const int cols = a.cols;
  const int nblocks = int((rows + P1_WG_ROWS - 1) / P1_WG_ROWS);
  if (blk >= nblocks) return;  // whole workgroup
  const int nchunk = (cols + P1_KC - 1) / P1_KC;
  const int grid1 = a.grid1;
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(a.A);
  const uint16_t* __restrict__ Bm = static_cast<const uint16_t*>(a.B);
  const uint8_t* __restrict__ X = static_cast<const uint8_t*>(a.X);
  uint8_t* __restrict__ R = static_cast<uint8_t*>(a.R);

  // X chunk c: rows [c*KC, c*KC + KC); thread t moves 16-B piece (t&7) of rows (t>>3) + 64q
  uint4 xr[2];
  auto load_x = [&](int c) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r = c * P1_KC + (tid >> 3) + 64 * q;
      xr[q] = r < cols ? ld16(X + size_t(r) * (K * 2) + (tid & 7) * 16) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
      *reinterpret_cast<uint4*>(&xs[buf][((tid >> 3) + 64 * q) * P1_XS + (tid & 7) * 16]) = xr[q];
  };
  // A operand fragments of chunk c of row block rbx: F[k-step][row tile]
  typedef bf16x8 Frags[4][2];
  auto load_a = [&](Frags& F, int rbx, int c) {
    const uint16_t* p[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      int64_t r = int64_t(rbx) * P1_WG_ROWS + wave * 32 + 16 * m + i;
      r = r < rows ? r : rows - 1;
      p[m] = A + r * a.lda + 8 * g + c * P1_KC;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
      if (c * P1_KC + 32 * s < cols)  // wave-uniform (cols % 32 == 0)
#pragma unroll
        for (int m = 0; m < 2; ++m) F[s][m] = __builtin_bit_cast(bf16x8, ld16_nt(p[m] + 32 * s));
  };

  f32x4 acc[2][4];
  auto zero_acc = [&]() {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  // R = acc - B, split hi/lo, into the k-packed layout: entry (row/8, iterate) = 32 B =
  // hi[8] | lo[8] (element row%8).  This lane holds rows row_w+16m+4g+r, iterate 16t+i.
  auto epilogue = [&](int rbx) {
    const int64_t row_w = int64_t(rbx) * P1_WG_ROWS + wave * 32;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
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
  };

  int rb = blk, c = 0, cur = 0;
  Frags FA, FB;
  load_x(0);
  load_a(FA, rb, 0);
  store_x(0);
  zero_acc();
  __syncthreads();
  // one chunk: prefetch the next chunk's A fragments and X rows, compute this chunk from
  // registers + LDS, publish the next X chunk, and finish the row block after its last chunk
  auto step = [&](Frags& F, Frags& N) -> bool {
    int rbn = rb, cn = c + 1;
    if (cn == nchunk) {
      cn = 0;
      rbn = rb + grid1;
    }
    const bool more = rbn < nblocks;
    if (more) {
      load_a(N, rbn, cn);
      load_x(cn);
    }
    const uint8_t* tile = xs[cur];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (c * P1_KC + 32 * s >= cols) break;  // wave-uniform
      bf16x8 bf[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) bf[t] = tr_operand(tile, P1_XS, 32 * s, 32 * t, lane);
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[m][t] = mfma(F[s][m], bf[t], acc[m][t]);
    }
    if (more) store_x(cur ^ 1);
    __syncthreads();
    cur ^= 1;
    if (rbn != rb) {
      epilogue(rb);
      zero_acc();
    }
    rb = rbn;
    c = cn;
    return more;
  };
  while (step(FA, FB) && step(FB, FA)) {
  }
}

// ---------------------------------------------------------------------------------------
// pass 1, cols <= 2048 (the c5 shape): split K over the 8 waves of the workgroup so the
// workgroup streams WHOLE rows.  Wave w owns columns [256w, 256w + 256) and holds that
// slice of X in registers for the whole kernel (8 k-steps x 4 iterate tiles of MFMA B
// operand = 128 VGPRs, transposed once through LDS); per block of 16 rows it reads
// A[16 rows][its 256 columns] (the 8 waves together: 16 contiguous rows = 64 KiB), the
// next block's fragments already in flight, and the 8 partial residuals are summed in LDS
// in wave order.  The chunked kernel above re-reads X per row block and walks every row in
// 256-B pieces 4 KiB apart, which left DRAM pages half used (3.3 TB/s, profiles/).
// pass-1 A loads: each instruction reads 64 B of 16 rows (the fragment layout), so the other
// half of every 128-B line is read by the wave's next instruction
#ifndef LSQB_P1_PROBE
#define LSQB_P1_PROBE 0
#endif
#ifndef LSQB_P1_LOAD
#define LSQB_P1_LOAD ld16
#endif
constexpr int Q_ROWS = 16;
constexpr int Q_KW = 256;                  // columns per wave
constexpr int Q_XS = K * 2 + 16;           // LDS bytes per staged X row
constexpr int Q_STAGE = 32 * Q_XS;         // one wave's staging window (one k-step of X)
constexpr int Q_PK = K + 4;                // partial-residual row stride (floats; conflict-free)
constexpr int Q_PART = Q_ROWS * Q_PK * 4;  // one wave's partial residual (fp32)

template <bool ARMED>
__global__ void __launch_bounds__(P1_THREADS) lsqb_resid_kernel(LsqbBatch batch) {
  constexpr int LDS = (8 * Q_STAGE > 8 * Q_PART ? 8 * Q_STAGE : 8 * Q_PART);
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];
  const int ti = task_of(batch.block1, batch.ntasks);
  const LsqbTask& a = batch.t[ti];
  const int blk = int(blockIdx.x) - batch.block1[ti];
  if constexpr (ARMED)  // device-armed (pass 2 follows on the stream)
    if (!wait_door(a.door, a.seq, batch.spin_ticks, batch.err)) return;
  if (disarmed(a.go, a.seq)) return;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t rows = a.rows;
  const int cols = a.cols;
  // blocks of 16 rows, an even count: pass 2 reads whole 32-row k-steps, zero past the end
  const int64_t nblocks = ((rows + 31) / 32) * 2;
  if (blk >= nblocks) return;  // whole workgroup
  const int grid1 = a.grid1;
  const int kc0 = wave * Q_KW;                       // first column of this wave
  const int nks = cols > kc0 ? ((cols - kc0) < Q_KW ? (cols - kc0) : Q_KW) / 32 : 0;  // its k-steps
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(a.A);
  const uint16_t* __restrict__ Bm = static_cast<const uint16_t*>(a.B);
  const uint8_t* __restrict__ X = static_cast<const uint8_t*>(a.X);
  uint8_t* __restrict__ R = static_cast<uint8_t*>(a.R);

  // this wave's X slice as MFMA B operands: XF[k-step][iterate tile]
  bf16x8 XF[8][4];
  uint8_t* stage = lds + wave * Q_STAGE;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
#pragma unroll
    for (int t = 0; t < 4; ++t) XF[s][t] = bf16x8{};  // k-steps past cols contribute A x 0
    if (s < nks) {
      // 32 X rows (4 KiB) -> the wave's window: lane moves 16-B pieces l, l+64, ..., l+192
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int piece = lane + 64 * q, r = piece >> 3, c16 = piece & 7;
        *reinterpret_cast<uint4*>(stage + r * Q_XS + c16 * 16) =
            ld16(X + size_t(kc0 + 32 * s + r) * (K * 2) + c16 * 16);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the window is written (one wave)
#pragma unroll
      for (int t = 0; t < 4; ++t) XF[s][t] = tr_operand(stage, Q_XS, 0, 32 * t, lane);
      __builtin_amdgcn_s_waitcnt(0xc07f);  // reads done before the window is rewritten
    }
  }
  __syncthreads();  // staging windows are reused as the partial-residual buffer below

  // Every load below is unconditional (row, k-step and block clamped to valid addresses,
  // their contributions zeroed by X = 0 / the row test at use): a load under a branch, or a
  // select between a fresh load and an old value, made the compiler wait for every load in
  // flight (s_waitcnt vmcnt(0)) before the MFMAs, which serialised the prefetch with the
  // compute (3.7 TB/s whatever the cache level).
  typedef bf16x8 Frags[8];
  const int kc_ok = kc0 < cols ? kc0 : 0;
  auto load_a = [&](Frags& F, int64_t rbx) {
    int64_t r = rbx * Q_ROWS + i;
    r = r < rows ? r : rows - 1;
    const uint16_t* p = A + r * a.lda + kc_ok + 8 * g;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int sc = s < nks ? s : 0;
      F[s] = __builtin_bit_cast(bf16x8, LSQB_P1_LOAD(p + 32 * sc));
    }
  };
  float* part = reinterpret_cast<float*>(lds);  // [wave][16 rows][64 iterates (+4 pad)]

  // this thread's reduction slot: (row group rg of 8 rows, iterate it, row pair h)
  const int it = tid & 63, h = (tid >> 6) & 3, rg = tid >> 8;
  // B of the slot's two rows of block rbx (prefetched with the block's A fragments)
  auto load_b = [&](uint16_t (&bv)[2], int64_t rbx) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      int64_t row = rbx * Q_ROWS + 8 * rg + 2 * h + e;
      row = row < rows ? row : rows - 1;  // rows past the end are zeroed at use
      bv[e] = Bm[row * K + it];
    }
  };

  int64_t rb = blk;
  Frags FA, FB;
  uint16_t BA[2], BB[2];
  load_a(FA, rb);
  load_b(BA, rb);
#if LSQB_P1_PROBE
  // measurement only (tools/gpu_p1_probe.sh, profiles/r01_lsqb_p1_probe.txt): 1 = the loads
  // alone, 2 = loads + MFMAs (no LDS reduction, no barriers); results feed a dead store
  float sink = 0.f;
#endif
  auto step = [&](Frags& F, Frags& N, uint16_t (&Bc)[2], uint16_t (&Bn)[2]) -> bool {
    const int64_t rbn = rb + grid1;
    const bool more = rbn < nblocks;
    const int64_t rbl = more ? rbn : rb;  // past the last block: re-read this one, unused
    load_a(N, rbl);
    load_b(Bn, rbl);
#if LSQB_P1_PROBE == 1
#pragma unroll
    for (int s = 0; s < 8; ++s) sink += float(F[s][0]) + float(F[s][7]);
    sink += float(Bc[0] ^ Bc[1]);
    rb = rbn;
    return more;
#endif
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = mfma(F[s], XF[s][t], acc[t]);
#if LSQB_P1_PROBE == 2
#pragma unroll
    for (int t = 0; t < 4; ++t) sink += acc[t][0] + acc[t][3];
    sink += float(Bc[0] ^ Bc[1]);
    rb = rbn;
    return more;
#endif
    // lane holds rows 4g + r, iterate 16t + i of this wave's partial
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(wave * Q_ROWS + 4 * g + r) * Q_PK + 16 * t + i] = acc[t][r];
    __syncthreads();
    // thread -> (row group rg of 8 rows, iterate it, row pair h): sum the 8 waves in order,
    // subtract B, split hi/lo, store 2 of the 8 rows of R8 entry (row/8, it)
    {
      uint32_t hi2 = 0, lo2 = 0;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int rl = 8 * rg + 2 * h + e;
        const int64_t row = rb * Q_ROWS + rl;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) v += part[(w * Q_ROWS + rl) * Q_PK + it];
        v = row < rows ? v - bf16_to_f32(Bc[e]) : 0.f;
        const uint16_t hv = bf16_rne(v), lv = bf16_rne(v - bf16_to_f32(hv));
        hi2 |= uint32_t(hv) << (16 * e);
        lo2 |= uint32_t(lv) << (16 * e);
      }
      uint8_t* ent = R + ((size_t((rb * Q_ROWS) / 8 + rg) * K + it) * 32) + 4 * h;
      *reinterpret_cast<uint32_t*>(ent) = hi2;
      *reinterpret_cast<uint32_t*>(ent + 16) = lo2;
    }
    __syncthreads();
    rb = rbn;
    return more;
  };
  while (step(FA, FB, BA, BB) && step(FB, FA, BB, BA)) {
  }
#if LSQB_P1_PROBE
  if (sink == 1234.5f && rows < 0) R[tid] = 1;
#endif
}

// ---------------------------------------------------------------------------------------
// pass 2: G = A^T R.  Workgroup (range rho, slice sigma): rows [32*s_begin, 32*s_end) x
// columns [256 sigma, 256 sigma + 256); wave w owns columns 64w..64w+63 of the slice and all
// 64 iterates (acc 4 x 4 tiles: G^T[iterate][column]).  Per k-step (32 rows) the A tile
// (32 x 256 bf16 = 16 KiB) is staged in LDS (double buffered) and read transposed as the B
// operand; R_hi / R_lo fragments are one 16-B load each.  Software pipeline: the tile of
// step s+2 and the R fragments of step s+1 are in flight while step s computes.
constexpr int P2_CW = 256;
constexpr int P2_AS = P2_CW * 2 + 16;
constexpr int P2_PART = K * P2_CW;  // floats per workgroup partial

__global__ void __launch_bounds__(kThreads, 2) lsqb_grad_kernel(LsqbBatch batch) {
  __shared__ __attribute__((aligned(16))) uint8_t as_[2][32 * P2_AS];
  __shared__ unsigned s_last;
  const int ti = task_of(batch.block2, batch.ntasks);
  const LsqbTask& a = batch.t[ti];
  const int blk = int(blockIdx.x) - batch.block2[ti];
  if (disarmed(a.go, a.seq)) return;
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
  // unconditional loads (see pass 1): columns past cols read column 0 and only feed G
  // columns that are never stored; steps past the range re-read its last step
  const int lc = c0 + 8 * (tid & 31) < cols ? c0 + 8 * (tid & 31) : 0;
  typedef uint4 Tile[4];
  typedef bf16x8 RFr[2][4];  // [hi, lo][iterate tile]
  auto load_tile = [&](Tile& T, int64_t s) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int64_t r = 32 * s + (tid >> 5) + 8 * q;
      r = r < rows ? r : rows - 1;  // rows past the end meet R = 0 (pass 1 zero-fills)
      T[q] = ld16_nt(A + r * a.lda + lc);
    }
  };
  auto store_tile = [&](const Tile& T, int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<uint4*>(&as_[buf][((tid >> 5) + 8 * q) * P2_AS + 16 * (tid & 31)]) = T[q];
  };
  auto load_r = [&](RFr& F, int64_t s) {
    const uint8_t* re = R + ((size_t(4 * s + g) * K + i) * 32);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      F[0][u] = __builtin_bit_cast(bf16x8, ld16(re + size_t(16 * u) * 32));
      F[1][u] = __builtin_bit_cast(bf16x8, ld16(re + size_t(16 * u) * 32 + 16));
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  Tile TA, TB;
  RFr RA, RB;
  int64_t s = s_begin;
  if (s < s_end) {
    load_tile(TA, s);
    load_tile(TB, s + 1 < s_end ? s + 1 : s_end - 1);
    load_r(RA, s);
    store_tile(TA, 0);
  }
  __syncthreads();
  int cur = 0;
  // step s: LDS buf[cur] holds tile s, Tn holds tile s+1 (in flight), Rc the R fragments of s
  auto step = [&](Tile& Tf, Tile& Tn, RFr& Rc, RFr& Rn) -> bool {
    if (s >= s_end) return false;
    load_tile(Tf, s + 2 < s_end ? s + 2 : s_end - 1);
    load_r(Rn, s + 1 < s_end ? s + 1 : s_end - 1);
    bf16x8 bf[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) bf[t] = tr_operand(as_[cur], P2_AS, 0, 2 * (64 * wave + 16 * t), lane);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[u][t] = mfma(Rc[0][u], bf[t], acc[u][t]);
        acc[u][t] = mfma(Rc[1][u], bf[t], acc[u][t]);
      }
    if (s + 1 < s_end) store_tile(Tn, cur ^ 1);
    __syncthreads();
    cur ^= 1;
    ++s;
    return true;
  };
  while (step(TA, TB, RA, RB) && step(TB, TA, RB, RA)) {
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
    if (old - a.tbase == unsigned(nslice - 1)) {
      publish_done(a.flag, a.seq);
      publish_peer(a.flag2, a.seq);
    }
  }
}

}  // namespace

hipError_t launch_lsqb(const LsqbBatch& a, hipStream_t s) {
  const int g1 = a.block1[a.ntasks], g2 = a.block2[a.ntasks];
  if (g1 <= 0 || g2 <= 0) return hipErrorInvalidValue;
  const bool armed = batch_armed(a);
  if (a.splitk && armed) hipLaunchKernelGGL(lsqb_resid_kernel<true>, dim3(g1), dim3(P1_THREADS), 0, s, a);
  else if (a.splitk) hipLaunchKernelGGL(lsqb_resid_kernel<false>, dim3(g1), dim3(P1_THREADS), 0, s, a);
  else if (armed) hipLaunchKernelGGL(lsqb_resid_chunked_kernel<true>, dim3(g1), dim3(P1_THREADS), 0, s, a);
  else hipLaunchKernelGGL(lsqb_resid_chunked_kernel<false>, dim3(g1), dim3(P1_THREADS), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(lsqb_grad_kernel, dim3(g2), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace mpa
