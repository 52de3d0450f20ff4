// Single-pass batched least squares by iterate halves, one wave per SIMD (BASELINE
// configs[4], "c5"):
//     G_i = A_i^T (A_i X - B_i)      A_i rows x cols bf16, X cols x 64 bf16, B_i rows x 64 bf16
// in the reference's compute slot (examples/iterative_example.jl:74 sleeps there), A read
// from HBM once.  The pair scheme of lsqp_kernel.hip (two workgroups on one XCD stream the
// same rows, member h owning iterates 32h .. 32h + 31; the second reader of a block finds it
// in L2), re-cut for the register file.
//
// Why one wave per SIMD.  The eight-wave cut (lsqp_kernel.hip) holds G (128 registers) and X
// (64) in a 256-register wave budget, so every LDS read of the block loop waits for itself
// (lgkmcnt(0) between reads) and the loop runs at ~2.3 us per 16-row block whether A comes
// from HBM or the Infinity Cache (profiles/r02_c5_lsqp_tuning.txt): issue-bound, not memory-
// bound.  Four waves of 512 registers each (G 256 accumulation registers, X 128, 128 free for
// the pipeline) let the reads of a phase run ahead of its MFMAs.
//
// Workgroup = 4 waves, one per SIMD, one workgroup per CU.  Wave w owns columns 512 w ..
// 512 w + 511 in both products:
//   X_h slice   [512 cols x 32 its] as MFMA B operands XF[k-step][iterate tile]      (128)
//   G partial   [512 cols x 32 its] fp32 accumulators G[iterate tile][column tile]   (256)
//   A slice     [16 rows x 512 cols] of each block, by the wave's own LDS-DMA (one 1-KiB
//               row per instruction) into a private 2-slot ring of 16 KiB slots, 16-B chunks
//               XOR-swizzled per row (swz below) so that the row reads of phase 1 and the
//               transposed reads of phase 2 are bank-conflict free
// Per block of 16 rows:
//   phase 1   P_w = A[rows, cols_w] X_h[cols_w, :]    16 x 32, split-K over the 4 waves
//   reduce    R = sum_w P_w (wave order) - B, bf16 hi + lo; each wave reduces a quarter  2 barriers
//   phase 2   G_w^T += R^T A[rows, cols_w]   one K = 32 MFMA per tile: k 0-15 the hi residual
//             of rows 0-15, k 16-31 the lo residual of the same rows; A^T by ds_read_b64_tr_b16
// The DMA of block u + 2 is issued once phase 2 of block u has read its slot.
//
// G over the row groups of a half: each wave's partial is stored write-through and summed
// by a fan-in-4 tree per (half, wave) in group order (the last arriver of a group carries it
// up); the root writes its 512 columns of G and the task's last slice publishes completion.
// Deterministic: fixed summation orders, no float atomics.
//
// MFMA maps (cdna_hip_programming.md §3), 16x16x32 bf16: A[m=i][k=8g+j], B[k=8g+j][n=i],
// C/D[m=4g+r][n=i]; lane l: i = l & 15, g = l >> 4.
#include <hip/hip_runtime.h>

#include "device_common.hpp"
#include "kernels.hpp"
#include "mpiasyncpools.h"

#ifndef MPA_MEASURE
#define MPA_MEASURE 0
#endif

namespace mpa {
namespace {

using namespace dev;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int K = kLsqbIterates;      // 64 iterates
constexpr int QW = 4;                 // waves per workgroup, one per SIMD
constexpr int QT = QW * 64;           // threads
constexpr int PRB = 16;               // rows per block
constexpr int QKW = 512;              // columns per wave
constexpr int ROWB = QKW * 2;         // bytes of one slice row (1 KiB)
constexpr int NKS = QKW / 32;         // k-steps of phase 1 (16)
constexpr int NCT = QKW / 16;         // column tiles of phase 2 (32)
constexpr int PH = 32;                // iterates per workgroup (one half)
constexpr int SLICE = PRB * ROWB;     // 16 KiB
constexpr int XS = PH * 2 + 16;       // X staging row stride (bytes)
constexpr int RS = 32 * 2 + 16;       // residual image row stride: k 0..31 bf16 + pad
constexpr int PF = 4;                 // G tree fan-in
static_assert(QW * QKW == kLsqpMaxCols, "4 waves x 512 columns");

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return uint16_t((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_f32(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }
__device__ __forceinline__ void lgkm_drain() { __builtin_amdgcn_s_waitcnt(0xc07f); }  // lgkmcnt(0)
// workgroup barrier that leaves the vector-memory queue alone (the next block's DMA stays in
// flight): LDS traffic drained, then s_barrier; the clobber pins LDS accesses on either side
__device__ __forceinline__ void barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA of one 1-KiB slice row: lane l's 16 B land at lds + 16 l.  Scalar base + 32-bit lane
// offset (the saddr form).  Inline asm on purpose, as in lsqp_kernel.hip: the compiler would
// guard every LDS read that may alias a DMA it knows of with vmcnt(0), waiting for the NEXT
// block too; the kernel orders its reads itself (vmcnt per block).
__device__ __forceinline__ void dma_row(const void* sbase, uint32_t voff, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(l)
               : "memory", "m0");
}
__device__ __forceinline__ void pf4(const void* src, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(l) : "memory", "m0");
}
__device__ __forceinline__ void dma16(const void* src, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(l) : "memory", "m0");
}

// 16-B chunk c of slice row r sits at chunk position c ^ swz(r) (bits 1-3 only, so 256-B
// groups of chunks stay put and k-steps / column tiles 4 (8) apart are immediate offsets)
__host__ __device__ constexpr int swz(int r) { return 2 * (r & 3) + (r & 8); }

// write-through 16-B store / load as two 8-B agent-scope accesses (the G tree's hand-off:
// MI355X_MICROARCH.md §inter-workgroup visibility, "one lane adds for the producer, the last
// adder loads")
__device__ __forceinline__ void st_wt(f32x4* p, const f32x4& v) {
  const unsigned long long* s = reinterpret_cast<const unsigned long long*>(&v);
  unsigned long long* d = reinterpret_cast<unsigned long long*>(p);
  __hip_atomic_store(d, s[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(d + 1, s[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ f32x4 ld_wt(const f32x4* p) {
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
  unsigned long long u[2];
  u[0] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  u[1] = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_bit_cast(f32x4, u);
}

__global__ void __launch_bounds__(QT, 1) lsqp4_kernel(LsqpBatch batch) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[QW][2][SLICE];
  __shared__ __attribute__((aligned(16))) uint8_t bring[2][PRB * PH * 2];
  __shared__ __attribute__((aligned(16))) f32x4 part[QW][2][64];
  __shared__ __attribute__((aligned(16))) uint8_t rimg[2 * 16 * RS];
  __shared__ __attribute__((aligned(16))) uint32_t sink[QW][64];

  // blocks b and b + 8 are the two halves of one pair (one XCD under round-robin placement;
  // speed only): pair index = (b / 16) * 8 + b % 8
  const int bx = int(blockIdx.x);
  const int h = (bx >> 3) & 1;
  const int pidx = (bx >> 4) * 8 + (bx & 7);
  if (pidx >= batch.grp0[batch.ntasks]) return;  // grid padding (whole workgroup)
  int ti = 0;
  while (ti + 1 < batch.ntasks && pidx >= batch.grp0[ti + 1]) ++ti;
  const LsqpTask& a = batch.t[ti];
  if (disarmed(a.go, a.seq)) return;  // every workgroup of the task alike
  const int q = pidx - batch.grp0[ti];
  const int ng = batch.grp0[ti + 1] - batch.grp0[ti];

  const int tid = threadIdx.x, lane = tid & 63, i = lane & 15, g = lane >> 4;
  const int qq = (lane >> 2) & 3, p4 = lane & 3;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t rows = a.rows;
  const int cols = a.cols;
  const int c0 = w * QKW;
  // valid k-steps of this wave; the loops always run all of them (k-steps past cols meet
  // X = 0, their G columns are never stored): branch-free block loop
  const int nks = cols > c0 ? ((cols - c0) < QKW ? (cols - c0) : QKW) / 32 : 0;
  const int64_t nblocks = (rows + PRB - 1) / PRB;
  const int64_t kb0 = nblocks * q / ng, kb1 = nblocks * (q + 1) / ng;
  const int nb = int(kb1 - kb0);
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(a.A);
  const uint16_t* __restrict__ Bm = static_cast<const uint16_t*>(a.B);
  const uint8_t* __restrict__ X = static_cast<const uint8_t*>(a.X);
  uint8_t* my0 = &ring[w][0][0];
  uint8_t* my1 = &ring[w][1][0];

  // ---- X_h slice -> XF, through the wave's two ring slots (32 KiB) in two rounds of eight
  // k-steps (32 X rows x 64 B each, row stride XS)
  bf16x8 XF[NKS][2];
#pragma unroll
  for (int rd = 0; rd < 2; ++rd) {
    uint4 xr[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int s = 8 * rd + (e >> 1), piece = lane + 64 * (e & 1), r = piece >> 2, c16 = piece & 3;
      xr[e] = s < nks ? *reinterpret_cast<const uint4*>(X + (size_t(c0 + 32 * s + r) * K + PH * h) * 2 + c16 * 16)
                      : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int piece = lane + 64 * (e & 1), r = piece >> 2, c16 = piece & 3;
      *reinterpret_cast<uint4*>(my0 + ((e >> 1) * 32 + r) * XS + c16 * 16) = xr[e];
    }
    lgkm_drain();
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        // rows 8g + qq (elements 0-3) and 8g + 4 + qq (4-7), iterate columns 16t + 4p4 .. +3
        const uint8_t* a0 = my0 + (s * 32 + 8 * g + qq) * XS + 2 * (16 * t) + 8 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * XS));
        XF[8 * rd + s][t] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    lgkm_drain();
  }

  // ---- the wave's DMA of block kb (clamped: past the range it re-reads the range's last
  // block into the free slot, unused, so every step issues the same number of loads).
  // Row e of the slice is one instruction; lane l loads logical chunk l ^ swz(e), stored at
  // position l.  Chunks past cols load column 0 (never used).
  const int64_t lda = a.lda;
  uint32_t voff[8];  // byte offset in the row, per distinct swizzle 2 * s8
#pragma unroll
  for (int s8 = 0; s8 < 8; ++s8) {
    const int c = lane ^ (2 * s8);
    voff[s8] = uint32_t(c0 + 8 * c < cols ? c0 + 8 * c : 0) * 2u;
  }
  const bool no_dma = MPA_MEASURE && (batch.dbg & 1), no_compute = MPA_MEASURE && (batch.dbg & 2);
  // phase probes (measurement build): 8 no phase 1, 16 no partials / reduce / barriers, 32 no phase 2
  const bool no_p1 = MPA_MEASURE && (batch.dbg & 8), no_red = MPA_MEASURE && (batch.dbg & 16),
             no_p2 = MPA_MEASURE && (batch.dbg & 32);
  auto dma = [&](int64_t kb, uint8_t* slot) __attribute__((always_inline)) {
    if (no_dma) return;
    const int64_t kc = kb < kb1 ? kb : (kb1 > kb0 ? kb1 - 1 : kb0);
    const int64_t r0 = kc * PRB;
    const uint16_t* p = A + r0 * lda;
    if (r0 + PRB <= rows) {  // every block but a ragged last one: one scalar add per row
#pragma unroll
      for (int e = 0; e < PRB; ++e) {
        dma_row(p, voff[swz(e) >> 1], slot + e * ROWB);
        p += lda;
      }
    } else {  // rows past the end re-read the last row (they meet R = 0)
      const int nv = int(rows - r0);
#pragma unroll
      for (int e = 0; e < PRB; ++e) dma_row(p + (e < nv ? e : nv - 1) * lda, voff[swz(e) >> 1], slot + e * ROWB);
    }
  };
  // L2 prefetch of block kb: 4 B per lane into a per-wave sink nobody reads, a lane per 128-B
  // line; member h takes rows 8h .. 8h + 7 of the wave's slice (the pair shares the XCD's L2),
  // so the DMA of the block, pfd steps later, finds its lines on chip
  const int pfd = batch.pfd;
  const uint32_t pfoff = uint32_t(c0 + 64 * (lane & 7) < cols ? c0 + 64 * (lane & 7) : 0) * 2u;
  auto pf = [&](int64_t kb) __attribute__((always_inline)) {
    if (no_dma) return;
    const int64_t kc = kb < kb1 ? kb : (kb1 > kb0 ? kb1 - 1 : kb0);
    int64_t row = kc * PRB + 8 * h + (lane >> 3);
    row = row < rows ? row : rows - 1;
    pf4(reinterpret_cast<const uint8_t*>(A + row * lda) + pfoff, &sink[w][0]);
  };
  // B of a block (16 rows x 32 iterates of half h = 16 x 64 B: one instruction of wave 0)
  const int brow = lane >> 2, bpiece = lane & 3;
  auto dma_b = [&](int64_t kb, uint8_t* bslot) __attribute__((always_inline)) {
    if (no_dma) return;
    const int64_t kc = kb < kb1 ? kb : (kb1 > kb0 ? kb1 - 1 : kb0);
    int64_t row = kc * PRB + brow;
    row = row < rows ? row : rows - 1;
    dma16(Bm + row * K + PH * h + 8 * bpiece, bslot);
  };

  f32x4 G[2][NCT];  // G^T tiles: [iterate tile][column tile], lane (i, g): its 4g + r, column i
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) G[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  // step u DMAs block u + 2 and prefetches block u + 2 + pfd.  The prologue issues what steps
  // -2 and -1 would have, so every step's wait counts the same loads; blocks 2 .. pfd - 1,
  // which no step prefetches, go first (older than everything the waits count)
  for (int d = 2; d < pfd; ++d) pf(kb0 + d);
  dma(kb0, my0);
  if (w == 0) dma_b(kb0, bring[0]);
  if (pfd) pf(kb0 + pfd);
  dma(kb0 + 1, my1);
  if (w == 0) dma_b(kb0 + 1, bring[1]);
  if (pfd) pf(kb0 + 1 + pfd);

  // LDS offsets inside a slot: k-step s reads chunk 4s + g of row i; column tile ct reads
  // chunks 2ct, 2ct + 1 of rows r0 and r0 + 4
  int off1[4], off2[8];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) off1[s4] = i * ROWB + ((4 * s4 + g) ^ swz(i)) * 16;
  {
    const int r0 = 8 * (g & 1) + qq;
#pragma unroll
    for (int c8 = 0; c8 < 8; ++c8) off2[c8] = r0 * ROWB + (((2 * c8) ^ swz(r0)) + (p4 >> 1)) * 16 + 8 * (p4 & 1);
  }
  // the reduce: wave w sums components 2 (w & 1), +1 of iterate tile w >> 1 (rows 4g + rr)
  const int rt = w >> 1, rc = 2 * (w & 1);

  auto step = [&](int u, uint8_t* slot, const uint8_t* bslot) __attribute__((always_inline)) {
    // this block's DMA has landed: all but the youngest loads (the next block's 16 rows and
    // wave 0's B piece) are done.  vmcnt(16) / vmcnt(17): expcnt / lgkmcnt fields left free
    if (pfd) {  // + the two prefetches issued after this block's DMA: vmcnt(18) / vmcnt(19)
      if (w == 0) __builtin_amdgcn_s_waitcnt(0x4F73);
      else __builtin_amdgcn_s_waitcnt(0x4F72);
    } else {
      if (w == 0) __builtin_amdgcn_s_waitcnt(0x4F71);
      else __builtin_amdgcn_s_waitcnt(0x4F70);
    }
    if (no_compute) {  // measurement: the DMA ring alone
      lgkm_drain();
      dma(kb0 + u + 2, slot);
      if (w == 0) dma_b(kb0 + u + 2, const_cast<uint8_t*>(bslot));
      if (pfd) pf(kb0 + u + 2 + pfd);
      return;
    }
    // ---- phase 1: P_w[rows 4g + r][iterate 16 t + i].  Fragment reads run eight k-steps
    // ahead of the MFMAs (the compiler waits for each with a counted lgkmcnt)
    constexpr int AD = 8;
    f32x4 p1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    if (!no_p1) {
    bf16x8 af[AD];
    auto rd1 = [&](int s) __attribute__((always_inline)) {
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(slot + off1[s & 3] + 256 * (s >> 2)));
    };
#pragma unroll
    for (int s = 0; s < AD; ++s) af[s] = rd1(s);
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      __builtin_amdgcn_sched_barrier(0);
      p1[0] = mfma(af[s % AD], XF[s][0], p1[0]);
      p1[1] = mfma(af[s % AD], XF[s][1], p1[1]);
      if (s + AD < NKS) af[s % AD] = rd1(s + AD);
    }
    __builtin_amdgcn_sched_barrier(0);
    }
    if (!no_red) {
    part[w][0][lane] = p1[0];
    part[w][1][lane] = p1[1];
    barrier();
    // ---- reduce: R = sum_w P_w - B for rows 4g + rc, +1 of iterate 16 rt + i, as hi / lo
    // into the phase-2 A-operand image rimg[t][i][k]: k = row (hi), 16 + row (lo)
    {
      f32x2 v = *reinterpret_cast<const f32x2*>(reinterpret_cast<const float*>(&part[0][rt][lane]) + rc);
#pragma unroll
      for (int ww = 1; ww < QW; ++ww)
        v += *reinterpret_cast<const f32x2*>(reinterpret_cast<const float*>(&part[ww][rt][lane]) + rc);
      const int64_t row0 = (kb0 + u) * PRB + 4 * g + rc;
      const uint32_t b2 = *reinterpret_cast<const uint32_t*>(bslot + (4 * g + rc) * (PH * 2) + 2 * (16 * rt + i));
      const uint32_t b3 = *reinterpret_cast<const uint32_t*>(bslot + (4 * g + rc + 1) * (PH * 2) + 2 * (16 * rt + i));
      uint32_t hw = 0, lw = 0;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float b = bf16_f32(uint16_t(e ? b3 : b2));
        const float x = row0 + e < rows ? v[e] - b : 0.f;  // rows past the end: R = 0
        const uint16_t hi = bf16_rne(x);
        const uint16_t lo = bf16_rne(x - bf16_f32(hi));
        hw |= uint32_t(hi) << (16 * e);
        lw |= uint32_t(lo) << (16 * e);
      }
      uint8_t* e = rimg + (rt * 16 + i) * RS + 2 * (4 * g + rc);
      *reinterpret_cast<uint32_t*>(e) = hw;
      *reinterpret_cast<uint32_t*>(e + 32) = lw;
    }
    barrier();
    }
    // ---- phase 2: G_w^T[it][col] += sum_k R-image[it][k] A[row(k)][col]
    bf16x8 RF[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
      RF[t] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(rimg + (t * 16 + i) * RS + 16 * g));
    // column tiles in chunks of 4 (8 transposed reads), double-buffered: the reads of chunk
    // c + 1 are issued before the MFMAs of chunk c
    constexpr int CH = 4;
    s16x4 tb[2][CH][2];
    auto rd = [&](int c, s16x4 (&d)[CH][2]) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int ct = CH * c + k;
        const uint8_t* src = slot + off2[ct & 7] + 256 * (ct >> 3);
        d[k][0] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src));
        d[k][1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src + 4 * ROWB));
      }
    };
    if (!no_p2) {
    rd(0, tb[0]);
#pragma unroll
    for (int c = 0; c < NCT / CH; ++c) {
      if (c + 1 < NCT / CH) rd(c + 1, tb[(c + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const bf16x8 bt =
            __builtin_bit_cast(bf16x8, __builtin_shufflevector(tb[c & 1][k][0], tb[c & 1][k][1], 0, 1, 2, 3, 4, 5, 6, 7));
        G[0][CH * c + k] = mfma(RF[0], bt, G[0][CH * c + k]);
        G[1][CH * c + k] = mfma(RF[1], bt, G[1][CH * c + k]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    }
    // the slot is read: DMA block u + 2 into it
    lgkm_drain();
    dma(kb0 + u + 2, slot);
    if (w == 0) dma_b(kb0 + u + 2, const_cast<uint8_t*>(bslot));
    if (pfd) pf(kb0 + u + 2 + pfd);
  };
  for (int u = 0; u < nb; u += 2) {
    step(u, my0, bring[0]);
    if (u + 1 < nb) step(u + 1, my1, bring[1]);
  }
  drain_vm();  // the trailing (unused) DMA pieces

  // ---- G over the row groups: fan-in-PF tree per (half, wave) of write-through partials
  const int nct = 2 * nks;
  const size_t wslab = size_t(2 * NCT) * 64;  // f32x4 units of one wave's partial
  f32x4* __restrict__ slab = static_cast<f32x4*>(a.slab) + (size_t(h) * kLsqpMaxGroups * QW + w) * wslab;
  const size_t qstride = size_t(QW) * wslab;  // between consecutive row groups
  uint32_t* ctr = a.ctr + (h * QW + w) * kLsqpCtrPerSlice;
  float* out = static_cast<float*>(a.out);
  auto store_out = [&](int t, int ct, const f32x4& v) __attribute__((always_inline)) {
    const int col = c0 + 16 * ct + i;
    if (ct < nct && col < cols)
      *reinterpret_cast<f32x4*>(out + size_t(col) * K + PH * h + 16 * t + 4 * g) = v;
  };
  if (ng == 1) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) store_out(t, ct, G[t][ct]);
  } else {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) st_wt(slab + size_t(q) * qstride + (t * NCT + ct) * 64 + lane, G[t][ct]);
    unsigned idx = unsigned(q), count = unsigned(ng), stride = 1;
    int lvl_off = 0, lvl_cap = (kLsqpMaxGroups + PF - 1) / PF;
    for (;;) {
      drain_vm();
      const unsigned first = (idx / PF) * PF;
      const unsigned gsize = count - first < unsigned(PF) ? count - first : unsigned(PF);
      unsigned old = 0;
      if (lane == 0) {
        uint32_t* c = &ctr[lvl_off + int(idx / PF)];
        old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == gsize) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      old = __shfl(old, 0, 64);
      if (old + 1 != gsize) return;  // an earlier arriver of the group: the last one carries it
      const unsigned next = (count + PF - 1) / PF;
      const f32x4* src = slab + size_t(first) * stride * qstride;
#pragma unroll 4
      for (int j2 = 0; j2 < 2 * NCT; ++j2) {
        const int j = j2 * 64 + lane;
        f32x4 s = ld_wt(src + j);
        for (unsigned m = 1; m < gsize; ++m) s += ld_wt(src + size_t(m) * stride * qstride + j);
        if (next == 1) store_out(j2 / NCT, j2 % NCT, s);
        else st_wt(slab + size_t(first) * stride * qstride + j, s);
      }
      if (next == 1) break;
      idx /= PF;
      count = next;
      stride *= PF;
      lvl_off += lvl_cap;
      lvl_cap = (lvl_cap + PF - 1) / PF;
    }
  }
  // this slice of G is written: the task's last slice (2 halves x 4 waves) publishes
  drain_vm();
  if (lane == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[2 * 8 * kLsqpCtrPerSlice], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == unsigned(2 * QW)) {
      __hip_atomic_store(&a.ctr[2 * 8 * kLsqpCtrPerSlice], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      publish_done(a.flag, a.seq);
    }
  }
}

}  // namespace

hipError_t launch_lsqp4(const LsqpBatch& a, hipStream_t s) {
  const int pairs = a.grp0[a.ntasks];
  if (pairs <= 0) return hipErrorInvalidValue;
  const int grid = (pairs + 7) / 8 * 16;
  hipLaunchKernelGGL(lsqp4_kernel, dim3(grid), dim3(QT), 0, s, a);
  return hipGetLastError();
}

}  // namespace mpa
