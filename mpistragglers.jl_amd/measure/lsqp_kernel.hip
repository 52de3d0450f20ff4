// Single-pass batched least squares by iterate halves (BASELINE configs[4], "c5"):
//     G_i = A_i^T (A_i X - B_i)      A_i rows x cols bf16, X cols x 64 bf16, B_i rows x 64 bf16
// placed in the reference's compute slot (examples/iterative_example.jl:74 sleeps there),
// with A read from HBM ONCE.
//
// Why halves.  The fp32 accumulator of G (cols x 64 x 4 B = 512 KiB at 2048 columns) is a
// whole CU's register file, so one workgroup cannot hold G while it streams full rows of A
// (which the residual needs).  Split the 64 iterates instead: a PAIR of workgroups streams
// the same rows, member h computing the residual and G for iterates 32h .. 32h + 31 only
// (R_h = A X_h - B_h needs full rows of A but only half of X; G_h = A^T R_h needs only R_h).
// No data moves between the members; the second to read a block of A finds it in the XCD's
// L2 (the members of a pair are placed on one XCD and start together), so HBM sees A once
// and the L2 -> CU stream twice (34.5 TB/s of L2 against 2 x ~7 TB/s).  The column-split
// alternative (lsqf_kernel.hip) exchanges partial residuals between CUs every block; the
// iterate-quarter one (lsqq, measurement build) reads A four times from L2.
//
// Workgroup = 8 waves, one per CU (2 waves per SIMD, <= 256 VGPRs).  Wave w owns columns
// 256 w .. 256 w + 255 in both products:
//   X_h slice   [256 cols x 32 its] as MFMA B operands, in registers for the kernel (64)
//   G partial   [256 cols x 32 its] fp32 MFMA accumulators (128)
//   A slice     [16 rows x 256 cols] of each block, streamed by the wave's OWN LDS-DMA into
//               a private 2-slot ring (8 KiB a slot; XOR-swizzled 16-B chunks so the row
//               reads of phase 1 and the transposed reads of phase 2 are bank-conflict free);
//               no other wave reads it, so the ring needs no barrier
// Per block of 16 rows:
//   phase 1   P_w = A[rows, cols_w] X_h[cols_w, :]          (16 x 32, split-K over the waves)
//   reduce    R = sum_w P_w (wave order) - B, as bf16 hi + lo (R = hi + lo to ~2^-17)   2 barriers
//   phase 2   G_w^T += R^T A[rows, cols_w]   one K = 32 MFMA per tile: k 0-15 the hi residual
//             of rows 0-15, k 16-31 the lo residual of the same rows; A^T by ds_read_b64_tr_b16
// The DMA of block u + 2 is issued as soon as phase 2 of block u has read its slot, so a
// block is in flight while the wave computes the one before it.
//
// G over the row groups of a half: each wave stores its partial write-through and a fan-in-4
// tree per (half, wave) sums them in group order (the last arriver of a group carries it up;
// nothing waits), the root writes its 256 columns of G and the task's last slice publishes
// completion.  Deterministic: fixed summation orders, no float atomics.
//
// MFMA maps (cdna_hip_programming.md §3), 16x16x32 bf16: A[m=i][k=8g+j], B[k=8g+j][n=i],
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
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int K = kLsqbIterates;    // 64 iterates
constexpr int PW = 8;               // waves per workgroup
constexpr int PT = PW * 64;         // threads
constexpr int PRB = 16;             // rows per block
constexpr int PKW = 256;            // columns per wave
constexpr int PH = 32;              // iterates per workgroup (one half)
constexpr int SLICE = PRB * PKW * 2;  // one wave's A slice of a block: 8 KiB (16 rows x 512 B)
constexpr int XS = PH * 2 + 16;     // X staging row stride (bytes)
constexpr int RS = 32 * 2 + 16;     // residual image row stride: k 0..31 bf16 + pad
constexpr int PF = 4;               // G tree fan-in

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return uint16_t((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_f32(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }
__device__ __forceinline__ void lgkm_drain() { __builtin_amdgcn_s_waitcnt(0xc07f); }  // lgkmcnt(0)
// workgroup barrier that leaves the vector-memory queue alone (the DMA of the next block stays
// in flight; __syncthreads' workgroup fences could wait for it): LDS traffic drained, then
// s_barrier; the memory clobber keeps the compiler from moving LDS accesses across it
__device__ __forceinline__ void barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA of 16 B per lane: lane l's bytes land at lds + 16 l (global_load_lds_dwordx4).  As
// inline asm on purpose: the compiler guards every LDS read that may alias an LDS-DMA it knows
// of with s_waitcnt vmcnt(0), which would also wait for the NEXT block's DMA and serialise
// the stream with the compute; the kernel orders its reads itself (vmcnt(8) per block, and
// each wave reads only what it loaded, or what crossed a barrier after the loader's wait).
__device__ __forceinline__ void dma16(const void* src, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(l) : "memory");
}

// L2 prefetch of 4 B per lane into a per-wave sink nobody reads (global_load_lds_dword): a
// lane per 128-B line of the wave's next-but-pfd slice brings the lines into the XCD's L2
// (and the Infinity Cache) well before the DMA asks for them, so a wave keeps HBM requests
// in flight beyond what its two 8-KiB LDS slots hold (MI355X_MICROARCH.md §Indexed rows: ~72
// KiB in flight per CU to hide an HBM miss; the ring gives one to two slots per wave)
__device__ __forceinline__ void pf4(const void* src, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(l) : "memory");
}

// 16-B chunk c (8 columns) of slice row r is stored at chunk position c ^ swz(r): distinct
// bank groups for the 16 rows a ds_read_b128 lane group touches (phase 1) and for the 8
// rows x 2 chunks a ds_read_b64_tr_b16 half-wave touches (phase 2)
__device__ __forceinline__ int swz(int r) { return 2 * (r & 3) + (r & 8); }

// write-through 16-B store / load as two 8-B agent-scope accesses (global_*_dwordx2 sc1):
// the hand-off protocol of the G tree (MI355X_MICROARCH.md §inter-workgroup visibility,
// "one lane adds for the producer, the last adder loads")
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

__global__ void __launch_bounds__(PT, 2) lsqp_kernel(LsqpBatch batch) {
  // each wave's two ring slots side by side (8 KiB apart: one address register reaches both
  // by immediate offsets), the B rows of the two blocks in flight, the phase-1 partials of
  // the 8 waves, the residual image of phase 2
  __shared__ __attribute__((aligned(16))) uint8_t ring[PW][2][SLICE];
  __shared__ __attribute__((aligned(16))) uint8_t bring[2][PRB * PH * 2];
  __shared__ __attribute__((aligned(16))) f32x4 part[PW][2][64];
  __shared__ __attribute__((aligned(16))) uint8_t rimg[2 * 16 * RS];
  __shared__ __attribute__((aligned(16))) uint32_t sink[PW][64];

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
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t rows = a.rows;
  const int cols = a.cols;
  const int c0 = w * PKW;
  // this wave's valid k-steps; the loop below always runs all 8 (and all 16 column tiles):
  // k-steps past cols meet X = 0 and their G columns are never stored, so the product loop
  // is branch-free (a partial last wave costs only MFMAs on the narrow test shapes)
  const int nks = cols > c0 ? ((cols - c0) < PKW ? (cols - c0) : PKW) / 32 : 0;
  const int nct = 2 * nks;
  const int64_t nblocks = (rows + PRB - 1) / PRB;
  const int64_t kb0 = nblocks * q / ng, kb1 = nblocks * (q + 1) / ng;
  const int nb = int(kb1 - kb0);
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(a.A);
  const uint16_t* __restrict__ Bm = static_cast<const uint16_t*>(a.B);
  const uint8_t* __restrict__ X = static_cast<const uint8_t*>(a.X);
  uint8_t* my0 = &ring[w][0][0];
  uint8_t* my1 = &ring[w][1][0];

  // ---- X_h slice -> MFMA B operands XF[k-step][iterate tile], through this wave's window
  // (32 X rows x 64 B per k-step; the window is slot 0 of its ring, not yet in use)
  bf16x8 XF[8][2];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    XF[s][0] = XF[s][1] = bf16x8{};  // k-steps past cols contribute A x 0
    if (s < nks) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int piece = lane + 64 * e, r = piece >> 2, c16 = piece & 3;
        *reinterpret_cast<uint4*>(my0 + r * XS + c16 * 16) =
            *reinterpret_cast<const uint4*>(X + (size_t(c0 + 32 * s + r) * K + PH * h) * 2 + c16 * 16);
      }
      lgkm_drain();
      const int qq = (lane >> 2) & 3, p4 = lane & 3;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        // rows 8g + qq (elements 0-3) and 8g + 4 + qq (4-7), iterate columns 16t + 4p4 .. +3
        const uint8_t* a0 = my0 + (8 * g + qq) * XS + 2 * (16 * t) + 8 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * XS));
        XF[s][t] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      lgkm_drain();
    }
  }

  // ---- the wave's DMA of block kb (clamped: past the range it re-reads the last block
  // into the free slot, unused, so every iteration issues the same number of loads)
  const int64_t lda = a.lda;
  auto dma = [&](int64_t kb, uint8_t* slot) __attribute__((always_inline)) {
    const int64_t kc = kb < kb1 ? kb : (kb1 > kb0 ? kb1 - 1 : kb0);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int r = 2 * e + (lane >> 5);  // 32 lanes per 512-B row
      int64_t row = kc * PRB + r;
      row = row < rows ? row : rows - 1;  // rows past the end meet R = 0
      const int c = (lane & 31) ^ swz(r);  // logical chunk stored at position lane & 31
      const int col = c0 + 8 * c < cols ? c0 + 8 * c : 0;  // columns past cols: unused
      dma16(A + row * lda + col, slot + e * 1024);
    }
  };
  // B of a block (16 rows x 32 iterates of half h = 16 x 64 B: ONE DMA instruction of wave 0)
  // lands beside the slot; the reducing waves read it from there
  const int brow = lane >> 2, bpiece = lane & 3;
  auto dma_b = [&](int64_t kb, uint8_t* bslot) __attribute__((always_inline)) {
    const int64_t kc = kb < kb1 ? kb : (kb1 > kb0 ? kb1 - 1 : kb0);
    int64_t row = kc * PRB + brow;
    row = row < rows ? row : rows - 1;
    dma16(Bm + row * K + PH * h + 8 * bpiece, bslot);
  };

  // the L2 prefetch of block kb: lane = (row lane / 4, 128-B line lane % 4) of the wave's slice
  const int pfd = batch.pfd;
  auto pf = [&](int64_t kb) __attribute__((always_inline)) {
    const int64_t kc = kb < kb1 ? kb : (kb1 > kb0 ? kb1 - 1 : kb0);
    int64_t row = kc * PRB + (lane >> 2);
    row = row < rows ? row : rows - 1;
    const int col = c0 + 64 * (lane & 3) < cols ? c0 + 64 * (lane & 3) : 0;
    pf4(A + row * lda + col, &sink[w][0]);
  };

  f32x4 G[2][16];  // G^T tiles: [iterate tile][column tile], lane (i, g): rows (its) 4g + r, column i
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ct = 0; ct < 16; ++ct) G[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the prologue issues what two earlier steps would have (DMA, B, prefetch pfd blocks ahead
  // of it), so every step's wait below counts the same loads; blocks 2 .. pfd - 1 are
  // prefetched first (older than everything the waits count)
  for (int d = 2; d < pfd; ++d) pf(kb0 + d);
  dma(kb0, my0);
  if (w == 0) dma_b(kb0, bring[0]);
  if (pfd) pf(kb0 + pfd);
  dma(kb0 + 1, my1);
  if (w == 0) dma_b(kb0 + 1, bring[1]);
  if (pfd) pf(kb0 + 1 + pfd);

  const int qq = (lane >> 2) & 3, p4 = lane & 3;
  // LDS offsets inside a slot (the swizzle of row r touches chunk bits 1-3 only, so k-steps
  // s and s + 4, and column tiles ct and ct + 8, are 256 B apart: immediate offsets)
  int off1[4], off2[8];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) off1[s4] = i * 512 + ((4 * s4 + g) ^ swz(i)) * 16;
  {
    const int r0 = 8 * (g & 1) + qq;
#pragma unroll
    for (int c8 = 0; c8 < 8; ++c8) off2[c8] = r0 * 512 + (((2 * c8) ^ swz(r0)) + (p4 >> 1)) * 16 + 8 * (p4 & 1);
  }
  // one block: slot / bv hold block u (static buffers: the loop below is unrolled by two)
  auto step = [&](int u, uint8_t* slot, const uint8_t* bslot) __attribute__((always_inline)) {
    // this block's DMA has landed: all but the youngest loads (the next block's 8 pieces,
    // wave 0's B piece, and with prefetch on the two prefetches issued after this block's
    // DMA) are done.  vmcnt(8 .. 11): expcnt / lgkmcnt fields left free
    if (pfd) {
      if (w == 0) __builtin_amdgcn_s_waitcnt(0x0F7B);
      else __builtin_amdgcn_s_waitcnt(0x0F7A);
    } else {
      if (w == 0) __builtin_amdgcn_s_waitcnt(0x0F79);
      else __builtin_amdgcn_s_waitcnt(0x0F78);
    }
    // ---- phase 1: P_w[rows 4g + r][iterate 16 t + i] over this wave's k-steps
    f32x4 p1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const bf16x8 af = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(slot + off1[s & 3] + 256 * (s >> 2)));
      p1[0] = mfma(af, XF[s][0], p1[0]);
      p1[1] = mfma(af, XF[s][1], p1[1]);
    }
    part[w][0][lane] = p1[0];
    part[w][1][lane] = p1[1];
    barrier();
    // ---- reduce (waves 0, 1 = iterate tiles 0, 1): R = sum_w P_w - B, hi / lo, into the
    // phase-2 A-operand image rimg[t][i][k]: k = row (hi), 16 + row (lo)
    if (w < 2) {
      f32x4 v = part[0][w][lane];
#pragma unroll
      for (int ww = 1; ww < PW; ++ww) {
        v += part[ww][w][lane];
        if (ww == 3) __builtin_amdgcn_sched_barrier(0);  // at most four partials in flight
      }
      const int64_t row0 = (kb0 + u) * PRB + 4 * g;
      uint16_t hi[4], lo[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint16_t b = *reinterpret_cast<const uint16_t*>(bslot + (4 * g + r) * (PH * 2) + 2 * (16 * w + i));
        const float x = row0 + r < rows ? v[r] - bf16_f32(b) : 0.f;
        hi[r] = bf16_rne(x);
        lo[r] = bf16_rne(x - bf16_f32(hi[r]));
      }
      uint8_t* e = rimg + (w * 16 + i) * RS;
      *reinterpret_cast<uint2*>(e + 8 * g) =
          make_uint2(uint32_t(hi[0]) | (uint32_t(hi[1]) << 16), uint32_t(hi[2]) | (uint32_t(hi[3]) << 16));
      *reinterpret_cast<uint2*>(e + 32 + 8 * g) =
          make_uint2(uint32_t(lo[0]) | (uint32_t(lo[1]) << 16), uint32_t(lo[2]) | (uint32_t(lo[3]) << 16));
    }
    barrier();
    // ---- phase 2: G_w^T[it][col] += sum_k R-image[it][k] A[row(k)][col]
    bf16x8 RF[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
      RF[t] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(rimg + (t * 16 + i) * RS + 16 * g));
#pragma unroll
    for (int ct = 0; ct < 16; ++ct) {
      // rows 8 (g & 1) + qq and + 4 (the same swizzle, 2 KiB further), columns 16 ct + 4 p4 ..
      const uint8_t* src = slot + off2[ct & 7] + 256 * (ct >> 3);
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src + 4 * 512));
      const bf16x8 bt = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      G[0][ct] = mfma(RF[0], bt, G[0][ct]);
      G[1][ct] = mfma(RF[1], bt, G[1][ct]);
      // a few column tiles of transposed reads in flight at a time: registers, not latency,
      // are the scarce resource here (G holds 128 of them)
      if ((ct & 3) == 3) __builtin_amdgcn_sched_barrier(0);
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
  const size_t wslab = size_t(32) * 64;  // f32x4 units of one wave's partial
  f32x4* __restrict__ slab = static_cast<f32x4*>(a.slab) + (size_t(h) * kLsqpMaxGroups * PW + w) * wslab;
  const size_t qstride = size_t(PW) * wslab;  // between consecutive row groups
  uint32_t* ctr = a.ctr + (h * PW + w) * kLsqpCtrPerSlice;
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
      for (int ct = 0; ct < 16; ++ct) store_out(t, ct, G[t][ct]);
  } else {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ct = 0; ct < 16; ++ct) st_wt(slab + size_t(q) * qstride + (t * 16 + ct) * 64 + lane, G[t][ct]);
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
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ct = 0; ct < 16; ++ct) {
          const int j = (t * 16 + ct) * 64 + lane;
          f32x4 s = ld_wt(src + j);
          for (unsigned m = 1; m < gsize; ++m) s += ld_wt(src + size_t(m) * stride * qstride + j);
          if (next == 1) store_out(t, ct, s);
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
  // this slice of G is written: the task's last slice (2 halves x 8 waves) publishes
  drain_vm();
  if (lane == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[2 * PW * kLsqpCtrPerSlice], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == unsigned(2 * PW)) {
      __hip_atomic_store(&a.ctr[2 * PW * kLsqpCtrPerSlice], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      publish_done(a.flag, a.seq);
    }
  }
}

}  // namespace

hipError_t launch_lsqp(const LsqpBatch& a, hipStream_t s) {
  const int pairs = a.grp0[a.ntasks];
  if (pairs <= 0) return hipErrorInvalidValue;
  const int grid = (pairs + 7) / 8 * 16;
  hipLaunchKernelGGL(lsqp_kernel, dim3(grid), dim3(PT), 0, s, a);
  return hipGetLastError();
}

}  // namespace mpa
