// Single-pass batched least squares by COLUMN pairs (BASELINE configs[4], "c5"):
//     G_i = A_i^T (A_i X - B_i)      A_i rows x cols bf16, X cols x 64 bf16, B_i rows x 64 bf16
// in the reference's compute slot (examples/iterative_example.jl:74 sleeps there), A read
// from HBM once and into each CU once.
//
// Why column pairs.  The iterate-halves pair (lsqp4_kernel.hip) has both members of a pair
// ingest every 64-KiB block of A (L2 -> LDS carries twice the unique bytes) into a 2-slot
// ring of 64-KiB slots: one block of read-ahead, so a block costs (compute + DMA round trip)
// / 2 (profiles/r02_c5_lsqp_tuning.txt).  Here the members split the COLUMNS: member h owns
// columns 1024 h .. 1024 h + 1023 with all 64 iterates (G: 1024 x 64 fp32 = the same 256
// registers per wave), ingests only its 32 KiB of each block, and the LDS holds a 4-slot
// ring, three blocks of read-ahead.  The price is one exchange per block: the members' partial
// products P_h = A[rows, cols_h] X[cols_h, :] (16 x 64 fp32) are summed into the residual.
//
// Workgroup = 4 waves, one per SIMD, one workgroup per CU.  Wave w computes on columns
// c0 = 1024 h + 256 w .. c0 + 255:
//   X slice   [256 cols x 64 its] as MFMA B operands XF[k-step][iterate tile]        (128)
//   G partial [256 cols x 64 its] fp32 accumulators G[iterate tile][column tile]     (256)
// Roles in the block loop: waves 1 and 2 DMA the block (two 256-column sub-slices each, one
// instruction per two 512-B rows), wave 3 DMAs B, wave 0 polls the partner's granules (a
// wave's vmcnt is in order, so a poll must not queue behind read-ahead DMAs of its own).
// Per step u (block u's phase 1 was done a step earlier):
//   A   barrier (block u + 1 landed; every wave done with block u - 1) -> DMA block u + 3
//   P1  phase 1 of block u + 1: P_w = A[rows, cols_w] X[cols_w, :], 16 x 64, split-K over
//       the waves; partials via LDS (barrier B), wave w sums iterate tile w in wave order and
//       publishes it as {tag, value} granules (Guideline 16 R2: the data is the flag)
//   X   wave 0 has the partner's P(u) (polled at the top of the step) in LDS (barrier C);
//       wave w forms R = P_0 + P_1 - B (two terms: order-free) for tile w as bf16 hi + lo
//   P2  (barrier D) G_w^T += R^T A[rows, cols_w], one K = 32 MFMA per tile (hi rows 0-15,
//       lo rows 0-15 of the same rows), A^T by ds_read_b64_tr_b16
// G over the row groups: write-through partials, fan-in-4 tree per (member, wave), last
// arriver carries (lsqp4's tree); the task's last slice publishes completion.
// Deterministic: fixed summation orders, no float atomics.
//
// Liveness: a workgroup takes a ticket at start; tickets 2k and 2k + 1 form a pair, so a
// member only ever waits for a workgroup that has started, and at most one workgroup per
// launch waits for a partner that has not.  Every wait is bounded (spin_ticks, err bit 16).
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
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int K = kLsqbIterates;   // 64 iterates
constexpr int QW = 4;              // waves, one per SIMD
constexpr int QT = QW * 64;
constexpr int PRB = 16;            // rows per block
constexpr int CW = 256;            // columns per wave
constexpr int CM = QW * CW;        // columns per member
constexpr int ROWB = CW * 2;       // 512 B: a wave's part of one row
constexpr int SUB = PRB * ROWB;    // 8 KiB: a wave's sub-slice of one block
constexpr int SLOT = QW * SUB;     // 32 KiB per block
constexpr int NS = 4;              // ring slots
constexpr int NKS = CW / 32;       // 8 k-steps of phase 1
constexpr int NCT = CW / 16;       // 16 column tiles of phase 2
constexpr int NT = K / 16;         // 4 iterate tiles
constexpr int BROW = K * 2;        // 128 B of B per row
constexpr int BSLOT = PRB * BROW;  // 2 KiB
constexpr int XS = BROW + 16;      // X staging row stride
constexpr int RS = 32 * 2 + 16;    // residual image row stride: k 0..31 bf16 + pad
constexpr int XR = kLsqcXR;
constexpr int PF = 4;              // G tree fan-in
constexpr int DMA_W = 17;          // DMA instructions per block of waves 1 and 2 (16 of A, 1 of B)
static_assert(CM == kLsqcMemberCols && 2 * CM == kLsqpMaxCols, "4 waves x 256 columns per member");
static_assert(XR >= 4, "a member runs at most 3 blocks ahead of its partner's reads");

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return uint16_t((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_f32(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }
__device__ __forceinline__ void lgkm_drain() { __builtin_amdgcn_s_waitcnt(0xc07f); }  // lgkmcnt(0)
// workgroup barrier that leaves the vector-memory queue alone (read-ahead DMAs stay in flight)
__device__ __forceinline__ void barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// s_waitcnt vmcnt(N) (gfx9 encoding: vmcnt bits 3:0 and 15:14; expcnt / lgkmcnt left free)
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// LDS-DMA of 1 KiB: lane l's 16 B land at lds + 16 l.  Scalar base + 32-bit lane offset (the
// saddr form); inline asm so that the compiler does not guard LDS reads with vmcnt(0) for
// it (the kernel counts its DMAs itself, vm_wait above)
__device__ __forceinline__ void dma1k(const void* sbase, uint32_t voff, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(l) : "memory");
}
__device__ __forceinline__ void dma16(const void* src, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(l) : "memory");
}

// 16-B chunk c of a 512-B sub-slice row r sits at chunk position c ^ swz(r) (bits 1-3 only:
// conflict-free row reads in phase 1 and transposed reads in phase 2, as in lsqp4)
__device__ __forceinline__ void dma16_sc1(const void* src, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(l) : "memory");
}

__host__ __device__ constexpr int swz(int r) { return 2 * (r & 3) + (r & 8); }

// write-through 16-B store / load as two 8-B agent-scope accesses (the G tree's hand-off)
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

// LA: phase 1 runs LA blocks ahead of phase 2 (the exchange has LA steps to land; DMA read-ahead
// NS - 1 - LA blocks beyond the block phase 1 needs)
// PR: phase probes, compile-time (measurement build only): 1 no A DMA, 2 no exchange, 8 no
// phase-1 MFMAs, 32 no phase-2 MFMAs
template <int LA, int PR>
__global__ void __launch_bounds__(QT, 1) lsqc_kernel(LsqpBatch batch) {
  static_assert(LA >= 1 && LA <= 2, "lookahead");
  __shared__ __attribute__((aligned(16))) uint8_t ring[NS][SLOT];
  __shared__ __attribute__((aligned(16))) uint8_t bring[NS][BSLOT];
  __shared__ __attribute__((aligned(16))) f32x4 part[QW][NT][64];  // the residual image aliases it
  __shared__ __attribute__((aligned(16))) uint8_t gimg[NT * 64 * 4 * 8];  // the partner's granules of a block

  const int tid = threadIdx.x, lane = tid & 63, i = lane & 15, g = lane >> 4;
  const int qq = (lane >> 2) & 3, p4 = lane & 3;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);

  // ---- ticket -> (task, row group, member)
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(batch.tick, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t + 1 == gridDim.x) __hip_atomic_store(batch.tick, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *reinterpret_cast<int*>(gimg) = int(t);
  }
  __syncthreads();
  const int ticket = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const int*>(gimg));
  if (ticket >= batch.grp0[batch.ntasks]) return;  // cannot happen: grid = workgroups
  int ti = 0;
  while (ti + 1 < batch.ntasks && ticket >= batch.grp0[ti + 1]) ++ti;
  const LsqpTask& a = batch.t[ti];
  if (disarmed(a.go, a.seq)) return;  // every workgroup of the task alike
  // phase probes (measurement build): 1 no A DMA, 2 no exchange, 8 no phase-1 MFMAs, 32 no phase-2 MFMAs
  constexpr bool no_dma = PR & 1, no_x = PR & 2, no_p1 = PR & 8, no_p2 = PR & 32;
  constexpr bool no_pub = PR & 4, no_poll = PR & 16, count_polls = PR & 64, late_pub = PR & 128, dma_at_c = PR & 256;
  unsigned repolls = 0;
  const int P = a.parts;
  const bool xchg = P == 2 && !no_x;  // the members exchange partial products
  const int j = ticket - batch.grp0[ti];
  const int q = j / P, h = j % P;
  const int ng = (batch.grp0[ti + 1] - batch.grp0[ti]) / P;

  const int64_t rows = a.rows;
  const int cols = a.cols;
  const int c0 = CM * h + CW * w;
  const int nks = cols > c0 ? ((cols - c0) < CW ? (cols - c0) : CW) / 32 : 0;
  const int64_t nblocks = (rows + PRB - 1) / PRB;
  const int64_t kb0 = nblocks * q / ng, kb1 = nblocks * (q + 1) / ng;
  const int nb = int(kb1 - kb0);
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(a.A);
  const uint16_t* __restrict__ Bm = static_cast<const uint16_t*>(a.B);
  const uint8_t* __restrict__ X = static_cast<const uint8_t*>(a.X);
  const int64_t lda = a.lda;

  // ---- X slice -> XF through the wave's quarter of the ring, two rounds of four k-steps
  // (128 X rows x 128 B each, row stride XS)
  bf16x8 XF[NKS][NT];
  {
    uint8_t* stg = &ring[w][0];
#pragma unroll
    for (int rd = 0; rd < 2; ++rd) {
      uint4 xr[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int piece = lane + 64 * e, r = piece >> 3, c16 = piece & 7;
        const int s = 4 * rd + (r >> 5);
        xr[e] = s < nks ? *reinterpret_cast<const uint4*>(X + size_t(c0 + 128 * rd + r) * BROW + c16 * 16)
                        : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int piece = lane + 64 * e, r = piece >> 3, c16 = piece & 7;
        *reinterpret_cast<uint4*>(stg + r * XS + c16 * 16) = xr[e];
      }
      lgkm_drain();
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          // X rows (k) 8g + qq (elements 0-3) and 8g + 4 + qq (4-7), iterates 16t + 4p4 .. +3
          const uint8_t* a0 = stg + (s * 32 + 8 * g + qq) * XS + 2 * (16 * t) + 8 * p4;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * XS));
          XF[4 * rd + s][t] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
      lgkm_drain();
    }
  }
  __syncthreads();  // every wave done with its staging before the DMAs overwrite the ring

  // ---- DMA of block kb (clamped: past the range it re-reads the range's last block into the
  // free slot, unused, so every step issues the same number of loads).  Waves 1 and 2: two
  // sub-slices each, one instruction per row pair: lanes 0-31 row 2e, lanes 32-63 row 2e + 1,
  // lane l loading logical chunk (l & 31) ^ swz(row) into position l & 31.  Chunks past cols
  // load column 0 (never used).  Wave 3: B (16 rows x 128 B, two instructions).
  const int hi_row = lane >> 5, pos = lane & 31;
  const int cs0 = CM * h + CW * (w == 2 ? 2 : 0);  // first sub-slice's column base (waves 1, 2)
  const uint32_t row_b = hi_row ? uint32_t(lda) * 2u : 0u;
  // byte offset of this lane's chunk of sub-slice cs0 + CW k, row pair e, in its row
  auto coff = [&](int k, int e) __attribute__((always_inline)) {
    const int col = cs0 + CW * k + 8 * (pos ^ swz(2 * e + hi_row));
    return uint32_t(col < cols ? col : 0) * 2u;
  };
  const uint32_t boff = uint32_t((lane >> 3) * BROW + (lane & 7) * 16);
  auto dma = [&](int64_t kb, int slot) __attribute__((always_inline)) {
    const int64_t kc = kb < kb1 ? kb : (kb1 > kb0 ? kb1 - 1 : kb0);
    const int64_t r0 = kc * PRB;
    if (w == 1 || w == 2) {
      uint8_t* base = &ring[slot][0] + (w == 2 ? 2 * SUB : 0);
      // B rows 8 (w - 1) .. + 7: lane l row l / 8, 16-B piece l % 8
      const int eb = w - 1;
      if (r0 + PRB <= rows) {
        if (!no_dma) {
          const uint16_t* p = A + r0 * lda;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            dma1k(p, coff(0, e) + row_b, base + 2 * e * ROWB);
            dma1k(p, coff(1, e) + row_b, base + SUB + 2 * e * ROWB);
            p += 2 * lda;
          }
        }
        dma1k(Bm + (r0 + 8 * eb) * K, boff, &bring[slot][0] + eb * 1024);
      } else {  // a ragged last block: rows past the end re-read the last row (R = 0 there)
        const int nv = int(rows - r0);
        if (!no_dma) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int row = 2 * e + hi_row;
            const uint8_t* rp = reinterpret_cast<const uint8_t*>(A + (r0 + (row < nv ? row : nv - 1)) * lda);
            dma16(rp + coff(0, e), base + 2 * e * ROWB);
            dma16(rp + coff(1, e), base + SUB + 2 * e * ROWB);
          }
        }
        int64_t row = r0 + 8 * eb + (lane >> 3);
        row = row < rows ? row : rows - 1;
        dma16(Bm + row * K + 8 * (lane & 7), &bring[slot][0] + eb * 1024);
      }
    }
  };

  // LDS offsets inside a wave's sub-slice: k-step s reads chunk 4s + g of row i; column tile
  // ct reads chunks 2ct, 2ct + 1 of rows r0 and r0 + 4
  int off1[4], off2[8];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) off1[s4] = i * ROWB + ((4 * s4 + g) ^ swz(i)) * 16;
  {
    const int r0 = 8 * (g & 1) + qq;
#pragma unroll
    for (int c8 = 0; c8 < 8; ++c8) off2[c8] = r0 * ROWB + (((2 * c8) ^ swz(r0)) + (p4 >> 1)) * 16 + 8 * (p4 & 1);
  }

  // exchange granules: [q][member][XR][tile][lane][4] {tag, fp32}
  unsigned long long* __restrict__ xg = a.xg;
  auto gslot = [&](int mem, int u) __attribute__((always_inline)) {
    return xg + ((size_t(q) * 2 + mem) * XR + (u % XR)) * (NT * 64 * 4);
  };
  const uint32_t tag0 = uint32_t(a.seq) * 65536u + 1u;  // tag of block u: tag0 + u (never 0 for u < 65535)
  const unsigned long long ticks = batch.spin_ticks;
  bool failed = false;

  // phase 1 of block v on slot sl -> this wave's quarter of P_h (iterate tile w)
  auto phase1 = [&](int sl, f32x4& Qw) __attribute__((always_inline)) {
    const uint8_t* sub = &ring[sl][0] + w * SUB;
    constexpr int AD = 4;
    f32x4 p1[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) p1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 af[AD];
    auto rd1 = [&](int s) __attribute__((always_inline)) {
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sub + off1[s & 3] + 256 * (s >> 2)));
    };
#pragma unroll
    for (int s = 0; s < AD; ++s) af[s] = rd1(s);
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (!no_p1) p1[t] = mfma(af[s % AD], XF[s][t], p1[t]);
      if (s + AD < NKS) af[s % AD] = rd1(s + AD);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < NT; ++t) part[w][t][lane] = p1[t];
    barrier();  // B
    Qw = part[0][w][lane];
#pragma unroll
    for (int ww = 1; ww < QW; ++ww) Qw += part[ww][w][lane];
  };
  // wave 3 publishes block v's P_h, all four tiles (summed in wave order, as each wave's Qw)
  // as soon as phase 1 is reduced.  Wave 3 issues no other vector memory op in the block loop
  // and never waits on vmcnt there, so the write-through stores drain in the background
  auto pub_sum = [&](const f32x4& Q3, f32x4 (&ps)[NT]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      ps[t] = Q3;
      if (t != 3) {
        ps[t] = part[0][t][lane];
#pragma unroll
        for (int ww = 1; ww < QW; ++ww) ps[t] += part[ww][t][lane];
      }
    }
  };
  // ... and stores them later (after barrier D, under phase 2, so that the stores' issue,
  // which queues behind the block DMAs in the CU's memory pipeline, delays no barrier): lane's
  // granules (t, lane, 0..3) as two 16-B write-through stores (a torn 16-B store still leaves
  // whole 8-B {value, tag} granules, each checked by the reader)
  auto pub_store = [&](int v, const f32x4 (&ps)[NT]) __attribute__((always_inline)) {
    if (no_pub) return;
    const uint32_t tg = tag0 + uint32_t(v);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      unsigned long long* d = gslot(h, v) + (size_t(t) * 64 + lane) * 4;
      const u32x4 lo = u32x4{__float_as_uint(ps[t][0]), tg, __float_as_uint(ps[t][1]), tg};
      const u32x4 hi = u32x4{__float_as_uint(ps[t][2]), tg, __float_as_uint(ps[t][3]), tg};
      asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(d), "v"(lo) : "memory");
      asm volatile("global_store_dwordx4 %0, %1, off offset:16 sc1" ::"v"(d), "v"(hi) : "memory");
    }
  };
  // wave 0: the partner's granules of block u -> gimg by LDS-DMA (write-through loads: L1 may
  // hold an older copy of the slot), 8 x 1 KiB
  auto poll_issue = [&](int u) __attribute__((always_inline)) {
    if (no_poll) return;
    const uint8_t* src = reinterpret_cast<const uint8_t*>(gslot(1 - h, u)) + 16 * lane;
#pragma unroll
    for (int k = 0; k < 8; ++k) dma16_sc1(src + 1024 * k, gimg + 1024 * k);
  };
  // ... wait for it, re-polling until every tag is block u's (bounded)
  auto poll_wait = [&](int u) __attribute__((always_inline)) {
    if (no_poll) return;
    const uint32_t want = tag0 + uint32_t(u);
    const unsigned long long t0 = rt_now();
    for (unsigned k = 1;; ++k) {
      drain_vm();
      bool ok = true;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint4 v = *reinterpret_cast<const uint4*>(gimg + 1024 * e + 16 * lane);
        ok &= v.y == want && v.w == want;
      }
      if (__all(ok) || failed || no_pub) break;
      ++repolls;
      if ((k & 63) == 0 && rt_now() - t0 > ticks) {
        if (lane == 0) __hip_atomic_fetch_or(batch.err, 16u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        failed = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      poll_issue(u);
    }
  };

  f32x4 G[NT][NCT];  // G^T tiles: [iterate tile][column tile], lane (i, g): its 4g + r, column i
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) G[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: DMA blocks 0 .. NS - 2; phase 1 of blocks 0 .. LA - 1
#pragma unroll
  for (int k = 0; k < NS - 1; ++k) dma(kb0 + k, k);
  if (w == 1 || w == 2) vm_wait<(NS - 1 - LA) * DMA_W>();
  barrier();
  f32x4 Qs[LA];  // this wave's tile of P_h for blocks u .. u + LA - 1
#pragma unroll
  for (int k = 0; k < LA; ++k) {
    if (k) barrier();  // every wave done reducing the previous block's partials
    Qs[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (k < nb) {
      phase1(k % NS, Qs[k]);
      if (xchg && w == 3) {
        f32x4 ps[NT];
        pub_sum(Qs[k], ps);
        pub_store(k, ps);
      }
    }
  }

  uint8_t* rimg = reinterpret_cast<uint8_t*>(&part[0][0][0]);
  if (xchg && w == 0) poll_issue(0);
  for (int u = 0; u < nb; ++u) {
    const int sl = u % NS;
    const bool more = u + LA < nb;
    // A: block u + LA landed (the DMAs of blocks u + LA + 1 .. u + NS - 2 are younger; waves
    // 1-2 issue no other vector memory op)
    if (w == 1 || w == 2) vm_wait<(NS - 2 - LA) * DMA_W>();
    barrier();
    if (!dma_at_c) dma(kb0 + u + NS - 1, (u + NS - 1) % NS);
    f32x4 Qn = f32x4{0.f, 0.f, 0.f, 0.f};
    if (more) phase1((u + LA) % NS, Qn);
    f32x4 ps[NT];
    if (xchg && w == 3 && more) {
      pub_sum(Qn, ps);
      if (!late_pub) pub_store(u + LA, ps);
    }
    // wave 0 (no other vector memory op): the partner's P(u) in gimg
    if (xchg && w == 0) poll_wait(u);
    const f32x4 Qk = Qs[0];
#pragma unroll
    for (int k = 0; k + 1 < LA; ++k) Qs[k] = Qs[k + 1];
    Qs[LA - 1] = Qn;
    barrier();  // C: the partner's P in LDS; every wave done reading `part` (the image aliases it)
    if (dma_at_c) dma(kb0 + u + NS - 1, (u + NS - 1) % NS);
    {
      f32x4 v = Qk;
      if (xchg) {  // the partner's tile w: values of granules (w, lane, 0..3)
        const uint4 g0 = *reinterpret_cast<const uint4*>(gimg + (w * 64 + lane) * 32);
        const uint4 g1 = *reinterpret_cast<const uint4*>(gimg + (w * 64 + lane) * 32 + 16);
        v += f32x4{__uint_as_float(g0.x), __uint_as_float(g0.z), __uint_as_float(g1.x), __uint_as_float(g1.z)};
      }
      const uint8_t* bs = &bring[sl][0];
      const int64_t row0 = (kb0 + u) * PRB + 4 * g;
      uint32_t hw[2] = {0, 0}, lw[2] = {0, 0};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float b = bf16_f32(*reinterpret_cast<const uint16_t*>(bs + (4 * g + r) * BROW + 2 * (16 * w + i)));
        const float x = row0 + r < rows ? v[r] - b : 0.f;  // rows past the end: R = 0
        const uint16_t hi = bf16_rne(x);
        const uint16_t lo = bf16_rne(x - bf16_f32(hi));
        hw[r >> 1] |= uint32_t(hi) << (16 * (r & 1));
        lw[r >> 1] |= uint32_t(lo) << (16 * (r & 1));
      }
      // image[it][k]: k = row (hi), 16 + row (lo)
      uint8_t* e = rimg + (w * 16 + i) * RS + 2 * (4 * g);
      *reinterpret_cast<uint2*>(e) = make_uint2(hw[0], hw[1]);
      *reinterpret_cast<uint2*>(e + 32) = make_uint2(lw[0], lw[1]);
    }
    barrier();  // D
    // wave 0: every wave has read gimg: poll the partner's P(u + 1) now, a step ahead of its use
    // (its publish was LA - 1 steps before this one), under this step's phase 2
    if (xchg && w == 0 && u + 1 < nb) poll_issue(u + 1);
    if (late_pub && xchg && w == 3 && more) pub_store(u + LA, ps);
    // ---- phase 2: G_w^T[it][col] += sum_k R-image[it][k] A[row(k)][col]
    bf16x8 RF[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
      RF[t] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(rimg + (t * 16 + i) * RS + 16 * g));
    const uint8_t* sub = &ring[sl][0] + w * SUB;
    constexpr int CH = 2;
    s16x4 tb[2][CH][2];
    auto rd = [&](int c, s16x4 (&d)[CH][2]) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int ct = CH * c + k;
        const uint8_t* src = sub + off2[ct & 7] + 256 * (ct >> 3);
        d[k][0] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src));
        d[k][1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src + 4 * ROWB));
      }
    };
    rd(0, tb[0]);
#pragma unroll
    for (int c = 0; c < NCT / CH; ++c) {
      if (c + 1 < NCT / CH) rd(c + 1, tb[(c + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const bf16x8 bt =
            __builtin_bit_cast(bf16x8, __builtin_shufflevector(tb[c & 1][k][0], tb[c & 1][k][1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int t = 0; t < NT; ++t)
          if (!no_p2) G[t][CH * c + k] = mfma(RF[t], bt, G[t][CH * c + k]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  drain_vm();  // the trailing (unused) DMA pieces and the last granule stores
  if (count_polls && w == 0 && lane == 0 && ticket < 4)
    printf("lsqc ticket %d: %u re-polls over %d blocks\n", ticket, repolls, nb);

  // ---- G over the row groups: fan-in-PF tree per (member, wave) of write-through partials
  const int nct = 2 * nks;
  const size_t wslab = size_t(NT * NCT) * 64;  // f32x4 units of one wave's partial (64 KiB)
  f32x4* __restrict__ slab = static_cast<f32x4*>(a.slab) + (size_t(h) * kLsqpMaxGroups * QW + w) * wslab;
  const size_t qstride = size_t(QW) * wslab;
  uint32_t* ctr = a.ctr + (h * 8 + w) * kLsqpCtrPerSlice;
  float* out = static_cast<float*>(a.out);
  auto store_out = [&](int t, int ct, const f32x4& v) __attribute__((always_inline)) {
    const int col = c0 + 16 * ct + i;
    if (ct < nct && col < cols) *reinterpret_cast<f32x4*>(out + size_t(col) * K + 16 * t + 4 * g) = v;
  };
  if (ng == 1) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) store_out(t, ct, G[t][ct]);
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t)
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
      for (int j2 = 0; j2 < NT * NCT; ++j2) {
        const int jj = j2 * 64 + lane;
        f32x4 s = ld_wt(src + jj);
        for (unsigned m = 1; m < gsize; ++m) s += ld_wt(src + size_t(m) * stride * qstride + jj);
        if (next == 1) store_out(j2 / NCT, j2 % NCT, s);
        else st_wt(slab + size_t(first) * stride * qstride + jj, s);
      }
      if (next == 1) break;
      idx /= PF;
      count = next;
      stride *= PF;
      lvl_off += lvl_cap;
      lvl_cap = (lvl_cap + PF - 1) / PF;
    }
  }
  // this slice of G is written: the task's last slice (members x 4 waves) publishes
  drain_vm();
  if (lane == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[2 * 8 * kLsqpCtrPerSlice], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == unsigned(P * QW)) {
      __hip_atomic_store(&a.ctr[2 * 8 * kLsqpCtrPerSlice], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      publish_done(a.flag, a.seq);
    }
  }
}

}  // namespace

hipError_t launch_lsqc(const LsqpBatch& a, hipStream_t s) {
  const int wgs = a.grp0[a.ntasks];
  if (wgs <= 0 || !a.tick) return hipErrorInvalidValue;
#if MPA_MEASURE
#define MPA_LSQC_PROBE(pr)                                                                     \
  if (a.dbg == pr) {                                                                         \
    if (a.pfd == 2) hipLaunchKernelGGL((lsqc_kernel<2, pr>), dim3(wgs), dim3(QT), 0, s, a);  \
    else hipLaunchKernelGGL((lsqc_kernel<1, pr>), dim3(wgs), dim3(QT), 0, s, a);             \
    return hipGetLastError();                                                                \
  }
  MPA_LSQC_PROBE(1) MPA_LSQC_PROBE(2) MPA_LSQC_PROBE(3) MPA_LSQC_PROBE(40) MPA_LSQC_PROBE(42)
  MPA_LSQC_PROBE(43) MPA_LSQC_PROBE(8) MPA_LSQC_PROBE(32) MPA_LSQC_PROBE(4) MPA_LSQC_PROBE(16)
  MPA_LSQC_PROBE(20) MPA_LSQC_PROBE(64) MPA_LSQC_PROBE(128) MPA_LSQC_PROBE(256)
#undef MPA_LSQC_PROBE
#endif
  if (a.pfd == 2) hipLaunchKernelGGL((lsqc_kernel<2, 0>), dim3(wgs), dim3(QT), 0, s, a);
  else hipLaunchKernelGGL((lsqc_kernel<1, 0>), dim3(wgs), dim3(QT), 0, s, a);
  return hipGetLastError();
}

}  // namespace mpa
