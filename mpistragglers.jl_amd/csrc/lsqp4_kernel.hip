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
//   A slice     [16 rows x 512 cols] of each block, by the wave's own LDS-DMA into a private
//               2-slot ring of 16 KiB slots, each slot 8 strips of 64 columns (one DMA
//               instruction = 8 rows x 128 B of a strip), 16-B chunks XOR-swizzled per row
//               (sw below) so that the row reads of phase 1 and the transposed reads of
//               phase 2 are bank-conflict free
// Per block of 16 rows:
//   phase 1   P_w = A[rows, cols_w] X_h[cols_w, :]    16 x 32, split-K over the 4 waves
//   reduce    R = sum_w P_w (wave order; wave 0 starts from -B), bf16 hi + lo, one barrier: every
//             wave sums all of R and moves it into phase 2's operand layout by lane swaps
//   phase 2   G_w^T += R^T A[rows, cols_w]   one K = 32 MFMA per tile: k 0-15 the hi residual
//             of rows 0-15, k 16-31 the lo residual of the same rows; A^T by ds_read_b64_tr_b16
// The DMA of block u + 2 goes out strip by strip inside phase 2 of block u, as each strip's
// column tiles are read (the DMA issue runs beside MFMAs and a strip's lead is ~1.5 blocks of
// compute); phase 1 of a block waits for it strip by strip.
//
// G over the row groups of a half: each wave's partial is stored write-through and summed
// by a fan-in-4 tree per (half, wave) in group order (the last arriver of a group carries it
// up); the root writes its 512 columns of G and the task's last slice publishes completion.
// Deterministic: fixed summation orders, no float atomics.
//
// MFMA maps (cdna_hip_programming.md §3), 16x16x32 bf16: A[m=i][k=8g+j], B[k=8g+j][n=i],
// C/D[m=4g+r][n=i]; lane l: i = l & 15, g = l >> 4.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "device_common.hpp"
#include "kernels.hpp"
#include "mpiasyncpools.h"


namespace mpa {
namespace {

using namespace dev;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
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
#ifndef MPA_LSQP4_PF
#define MPA_LSQP4_PF 4                // G tree fan-in
#endif
constexpr int PF = MPA_LSQP4_PF;
static_assert(PF >= 2 && PF <= 8, "tree fan-in");
#ifndef MPA_LSQP4_TJB
#define MPA_LSQP4_TJB 8               // G tree: column tiles per round of loads (x PF members in flight)
#endif
constexpr int kTreeJB = MPA_LSQP4_TJB;
static_assert((2 * 32) % kTreeJB == 0, "tiles per round");
#ifndef MPA_LSQP4_P2L
#define MPA_LSQP4_P2L 1               // phase-2 transposed-read chunks in flight ahead (1 vs 2: -1 %, r02_c5_strip_ring.txt)
#endif
#ifndef MPA_LSQP4_AD
#define MPA_LSQP4_AD 3                // phase-1 fragment read-ahead in k-steps (3 beats 2, 4, 6)
#endif
static_assert(QW * QKW == kLsqpMaxCols, "4 waves x 512 columns");
static_assert(NKS == 16 && NCT == 32, "8 strips of 64 columns per wave");

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// MPA_LSQP4_PROBE (timing-probe builds only, wrong results: make BUILD=... EXTRA=-DMPA_LSQP4_PROBE=n,
// profiles/r03_c5_probes.txt): 1 no strip DMAs in the block loop, 2 no cross-wave exchange /
// barrier in the reduce, 4 no phase-1 MFMAs, 8 half the phase-2 LDS reads (r04_c5_pipelined.txt),
// 16 no L2 prefetch (r06: 1 | 16 = the loop with no memory traffic but B, profiles/r06_c5_prefetch_cu.txt),
// 32 no G tree (every wave stores its partial and goes to the publish: what the tree costs a launch)
#ifndef MPA_LSQP4_PROBE
#define MPA_LSQP4_PROBE 0
#endif
#ifndef MPA_LSQP4_P2I
#define MPA_LSQP4_P2I 1  // phase-2 reads interleaved with the MFMAs
#endif
#ifndef MPA_LSQP4_VACC
#define MPA_LSQP4_VACC 1  // phase-1 accumulators in VGPRs (inline asm MFMAs)
#endif
// Phase 1's accumulators in VGPRs.  G takes all 256 AGPRs, and the compiler gives every MFMA
// intrinsic AGPR accumulators, so with intrinsics it parks 8 G registers in VGPRs around every
// phase 1 (24 moves per block).  These asm forms keep the phase-1 chain in VGPRs.  Hazards are
// the kernel's (the compiler does not look inside): the chain reads its own previous result as
// SrcC (exact overlap: back to back is allowed), A / B operands come from LDS reads (lgkmcnt,
// which the compiler does insert for asm operands) or registers written long before; the one
// non-MFMA reader of the result gets 16 wait states first (mfma_v_settle)
__device__ __forceinline__ f32x4 mfma_v0(const bf16x8& a, const bf16x8& b) {
  f32x4 d;
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ void mfma_v(f32x4& d, const bf16x8& a, const bf16x8& b) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_v_settle(f32x4& d0, f32x4& d1) {
  asm volatile("s_nop 7\n\ts_nop 7" : "+v"(d0), "+v"(d1));
}
__device__ __forceinline__ void lgkm_drain() { __builtin_amdgcn_s_waitcnt(0xc07f); }  // lgkmcnt(0)
// lgkmcnt(N) alone (vmcnt / expcnt fields left free)
template <int N>
__device__ __forceinline__ void lgkm_wait() {
  static_assert(N >= 0 && N < 16, "lgkmcnt is 4 bits");
  __builtin_amdgcn_s_waitcnt(0xc07f | (N << 8));
}
// workgroup barrier that leaves the vector-memory queue alone (the next block's DMA stays in
// flight): LDS traffic drained, then s_barrier; the clobber pins LDS accesses on either side
__device__ __forceinline__ void barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA of one 1-KiB slice row: lane l's 16 B land at lds + 16 l.  Scalar base + 32-bit lane
// offset (the saddr form).  Inline asm on purpose, as in lsqp_kernel.hip: the compiler would
// guard every LDS read that may alias a DMA it knows of with vmcnt(0), waiting for the NEXT
// block too; the kernel orders its reads itself (vmcnt per block).
__device__ __forceinline__ void dma_row(const void* sbase, uint32_t voff, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(l) : "memory");
}
__device__ __forceinline__ void pf4(const void* src, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(l) : "memory");
}
__device__ __forceinline__ void dma16(const void* src, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(l) : "memory");
}
// the saddr forms with an immediate offset (FULL blocks): the instruction adds OFF to the
// global address AND to the LDS address (llvm.amdgcn.global.load.lds: "applied to both"), so
// m0 = LDS destination - OFF.  One scalar base per block instead of a 64-bit add per strip
// A whole strip (both halves) under one M0 write: half j lands at lds + 1024 j and reads its
// rows at voff_j, so with m0 = lds - OFF and offsets OFF and OFF + 1024 the second half's lane
// offset is passed as voff_1 - 1024 (voff_1 >= 8 rows >= 1024 B)
template <int OFF>
__device__ __forceinline__ void dma_strip_off(const void* sbase, uint32_t voff0, uint32_t voff1m, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds))) - uint32_t(OFF);
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %2 offset:%4\n\t"
               "global_load_lds_dwordx4 %1, %2 offset:%5"
               ::"v"(voff0), "v"(voff1m), "s"(sbase), "s"(l), "i"(OFF), "i"(OFF + 1024) : "memory");
}
__device__ __forceinline__ void dma16_s(const void* sbase, uint32_t voff, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(l) : "memory");
}
__device__ __forceinline__ void pf4_s(const void* sbase, uint32_t voff, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(voff), "s"(sbase), "s"(l) : "memory");
}

// 16-B chunk c of strip row r sits at chunk position c ^ sw(r) (bits 1-2 only: chunk pairs
// stay together); found by search over the linear maps of r's bits for conflict-free reads of
// both phases (tools/lsqp4_swizzle.py)
__host__ __device__ constexpr int sw(int r) { return 2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1); }

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

#if MPA_MEASURE
// In-kernel clock (measurement build only; MI355X_MICROARCH.md 'DVFS give-back' item 6): thread 0
// of every workgroup stamps s_memtime (shader cycles) and s_memrealtime (100 MHz) once before and
// once after its block loop, and its block count; the last launch of two or more tasks (the 7- and 8-task
// launches of the c5 loop, not the 1-task release after it) is read by lsqp4_clock_dump() (MPA_LSQP4_CLOCK=1,
// at comm teardown).  Nothing in the kernel reads them.
constexpr int kClockSlots = 4096;
__device__ unsigned long long g_lsqp4_clk[kClockSlots][5];
#endif

// FULL: every task of the batch has cols == 2048 and rows % 16 == 0 (BASELINE c5's shape):
// no ragged block, no partial strip, so the block loop drops the clamps, selects and masks
// of the general form and addresses a block from ONE scalar base (immediate strip offsets)
template <bool ARMED, bool FULL>
__global__ void __launch_bounds__(QT, 1) lsqp4_kernel(LsqpBatch batch) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[QW][2][SLICE];
  __shared__ __attribute__((aligned(16))) uint8_t bring[2][PRB * PH * 2];
  // phase-1 partials, double-buffered by block parity: with one barrier per block, a wave
  // may store block u + 1's partial while a slower wave still reads block u's
  __shared__ __attribute__((aligned(16))) f32x4 part[2][QW][2][64];
  __shared__ __attribute__((aligned(16))) uint32_t sink[QW][64];
  // zeros in B's slot layout, one per wave (each wave zeroes its own: no barrier): the -B MFMA
  // operand of waves 1-3 (MPA_LSQP4_VACC)
  __shared__ __attribute__((aligned(16))) uint8_t bzero[QW][PRB * PH * 2];

  // blocks b and b + 8 are the two halves of one pair (one XCD under round-robin placement;
  // speed only): pair index = (b / 16) * 8 + b % 8
  const int bx = int(blockIdx.x);
  const int h = (bx >> 3) & 1;
  const int pidx = (bx >> 4) * 8 + (bx & 7);
  if (pidx >= batch.grp0[batch.ntasks]) return;  // grid padding (whole workgroup)
  int ti = 0;
  while (ti + 1 < batch.ntasks && pidx >= batch.grp0[ti + 1]) ++ti;
  const LsqpTask& a = batch.t[ti];
  // a pre-armed task its server cancelled computes but neither writes G nor publishes: the
  // go word (host memory) is read once per writing wave at the end (disarmed() below), not by
  // every workgroup before any work (profiles/r02_arm_go_word.txt)
  const int q = pidx - batch.grp0[ti];
  const int ng = batch.grp0[ti + 1] - batch.grp0[ti];
  if constexpr (ARMED)
    if (!wait_door(a.door, a.seq, batch.spin_ticks, batch.err)) return;  // device-armed

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
  // wave-uniform by construction; readfirstlane keeps the block arithmetic on the scalar unit
  // block indices in 32 bits (SALU has no 64-bit compare): the clamps below stay scalar
  const int kb0 = __builtin_amdgcn_readfirstlane(int(nblocks * q / ng)),
            kb1 = __builtin_amdgcn_readfirstlane(int(nblocks * (q + 1) / ng));
  const int kblast = kb1 > kb0 ? kb1 - 1 : kb0;  // past the range, DMAs re-read this block
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
  *reinterpret_cast<uint4*>(&bzero[w][16 * lane]) = make_uint4(0, 0, 0, 0);
  lgkm_drain();

  // ---- the wave's DMA of block kb (clamped: past the range it re-reads the range's last
  // block into the free slot, unused, so every step issues the same number of loads)
  const int64_t lda = a.lda;
  // ---- the strip ring.  A wave's slice of a block (16 rows x 512 columns) is 8 strips of 64
  // columns; strip k (2 KiB) sits at k * 2048, row r of it (128 B) at r * 128, logical 16-B
  // chunk c of the row at position c ^ sw(r): bank-conflict free for phase 1's row reads and
  // phase 2's transposed reads.  One DMA instruction moves half a strip (8 rows x 128 B; lane l:
  // row 8j + l / 8, position l % 8), so phase 2 hands a strip back as soon as its four column
  // tiles are read, and phase 1 waits for a block strip by strip.
  // Per-lane offsets from the block's first row at column c0: strip half j, a full strip or
  // one whose last 32 columns lie past cols (cols % 32 == 0; those lanes re-read the first 32)
  uint32_t vfull[2], vpart[2];
  auto voffs = [&](int nv, uint32_t (&vf)[2], uint32_t (&vp)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pr = 8 * j + (lane >> 3);     // row position in the strip
      const int rr = pr < nv ? pr : nv - 1;   // rows past the end re-read the last row (R = 0)
      const int c = (lane & 7) ^ sw(pr);
      const uint32_t rb = uint32_t(rr) * uint32_t(lda) * 2u;
      vf[j] = rb + uint32_t(c) * 16u;
      vp[j] = rb + uint32_t(c & 3) * 16u;
    }
  };
  voffs(PRB, vfull, vpart);
  struct Blk {
    const uint16_t* p;  // first row of the block (clamped into the range)
    int nv;             // valid rows
  };
  auto blk = [&](int kb) __attribute__((always_inline)) {
    const int kc = kb < kb1 ? kb : kblast;
    const int64_t r0 = int64_t(kc) * PRB;
    return Blk{A + r0 * lda, int(rows - r0 < PRB ? rows - r0 : PRB)};
  };
  // strip k of a block into a slot: 2 instructions.  Strips wholly past cols load columns
  // 0 .. 31 (finite data that meets X = 0; their G columns are never stored)
  auto dma_strip = [&](const Blk& b, const uint32_t (&vf)[2], const uint32_t (&vp)[2], int k, uint8_t* slot)
      __attribute__((always_inline)) {
    if constexpr (FULL) {
      // every strip of every block lies inside the rows: base = the block's first row at c0,
      // strip k at the immediate offset 128 k (k is a constant once the loops are unrolled)
      const uint16_t* base = b.p + c0;
      const uint32_t v1m = vf[1] - 1024u;
      uint8_t* d = slot + 2048 * k;
      switch (k) {
        case 0: dma_strip_off<0>(base, vf[0], v1m, d); break;
        case 1: dma_strip_off<128>(base, vf[0], v1m, d); break;
        case 2: dma_strip_off<256>(base, vf[0], v1m, d); break;
        case 3: dma_strip_off<384>(base, vf[0], v1m, d); break;
        case 4: dma_strip_off<512>(base, vf[0], v1m, d); break;
        case 5: dma_strip_off<640>(base, vf[0], v1m, d); break;
        case 6: dma_strip_off<768>(base, vf[0], v1m, d); break;
        default: dma_strip_off<896>(base, vf[0], v1m, d); break;
      }
    } else {
      const int cb = c0 + 64 * k;
      const bool full = cb + 64 <= cols;
      const uint16_t* base = b.p + (cb < cols ? cb : 0);
#pragma unroll
      for (int j = 0; j < 2; ++j) dma_row(base, full ? vf[j] : vp[j], slot + 2048 * k + 1024 * j);
    }
  };
  auto dma = [&](int kb, uint8_t* slot) __attribute__((always_inline)) {
    const Blk b = blk(kb);
    uint32_t vf[2], vp[2];
    voffs(b.nv, vf, vp);
#pragma unroll
    for (int k = 0; k < 8; ++k) dma_strip(b, vf, vp, k, slot);
  };
  // L2 prefetch of block kb: 4 B per lane into a per-wave sink nobody reads, a lane per 128-B
  // line; member h takes rows 8h .. 8h + 7 of the wave's slice (the pair shares the XCD's L2),
  // so the DMA of the block, pfd steps later, finds its lines on chip.  Always issued (pfd = 0
  // re-touches the block being loaded), so every wait counts the same loads
  const int pfd = batch.pfd;
  const uint32_t pfoff = uint32_t(c0 + 64 * (lane & 7) < cols ? c0 + 64 * (lane & 7) : 0) * 2u;
  const uint32_t pfv = uint32_t(lane >> 3) * uint32_t(lda) * 2u + pfoff;  // FULL: lane offset from row 8h
  auto pf = [&](int kb) __attribute__((always_inline)) {
    const int kc = kb < kb1 ? kb : kblast;
    if constexpr (FULL) {
      pf4_s(A + (int64_t(kc) * PRB + 8 * h) * lda, pfv, &sink[w][0]);
    } else {
      int64_t row = int64_t(kc) * PRB + 8 * h + (lane >> 3);
      row = row < rows ? row : rows - 1;
      pf4(reinterpret_cast<const uint8_t*>(A + row * lda) + pfoff, &sink[w][0]);
    }
  };
  // B of a block (16 rows x 32 iterates of half h = 16 x 64 B): one instruction of wave 0; the
  // other waves touch the same rows into their sink instead, so every wave counts one load
  const int brow = lane >> 2, bpiece = lane & 3;
  const uint32_t bv = uint32_t(brow * K + 8 * bpiece) * 2u;  // FULL: lane offset from the block's first B row
  auto dma_b = [&](int kb, uint8_t* bslot) __attribute__((always_inline)) {
    const int kc = kb < kb1 ? kb : kblast;
    if constexpr (FULL) {
      const uint16_t* sb = Bm + int64_t(kc) * PRB * K + PH * h;
      if (w == 0) dma16_s(sb, bv, bslot);
      else pf4_s(sb, bv, &sink[w][0]);
    } else {
      int64_t row = int64_t(kc) * PRB + brow;
      row = row < rows ? row : rows - 1;
      const uint16_t* src = Bm + row * K + PH * h + 8 * bpiece;
      if (w == 0) dma16(src, bslot);
      else pf4(src, &sink[w][0]);
    }
  };
  // vmcnt(n) alone (expcnt / lgkmcnt fields left free)
#define MPA_VMCNT(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (((n) >> 4) << 14) | 0x0F70)
  // strip k of the current block has landed once at most the loads issued after it are
  // pending: the rest of the block's strips (2 (7 - k)), its prefetch, and the next block's B,
  // 16 strip loads and prefetch (18).  k is a constant after unrolling: one wait survives
  auto wait_strip = [&](int k) __attribute__((always_inline)) {
    switch (k) {
      case 0: MPA_VMCNT(2 * 7 + 19); break;
      case 1: MPA_VMCNT(2 * 6 + 19); break;
      case 2: MPA_VMCNT(2 * 5 + 19); break;
      case 3: MPA_VMCNT(2 * 4 + 19); break;
      case 4: MPA_VMCNT(2 * 3 + 19); break;
      case 5: MPA_VMCNT(2 * 2 + 19); break;
      case 6: MPA_VMCNT(2 * 1 + 19); break;
      default: MPA_VMCNT(19); break;
    }
  };

  f32x4 G[2][NCT];  // G^T tiles: [iterate tile][column tile], lane (i, g): its 4g + r, column i
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) G[t][ct] = f32x4{0.f, 0.f, 0.f, 0.f};

  // step u issues block u + 2: B, its 8 strips (inside phase 2, as block u's strips are read),
  // then the prefetch of block u + 2 + pfd.  The prologue issues what steps -2 and -1 would
  // have, so every wait counts the same loads; blocks 2 .. pfd - 1, which no step prefetches,
  // go first (older than everything the waits count)
  for (int d = 2; d < pfd; ++d) pf(kb0 + d);
  dma_b(kb0, bring[0]);
  dma(kb0, my0);
  pf(kb0 + pfd);
  dma_b(kb0 + 1, bring[1]);
  dma(kb0 + 1, my1);
  pf(kb0 + 1 + pfd);

  // LDS offsets inside a slot: k-step s reads chunk 4 (s & 1) + g of row i of strip s / 2;
  // column tile ct reads chunks 2 (ct & 3), +1 of rows r0 and r0 + 4 of strip ct / 4
  int off1[2], off2[4];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) off1[s2] = i * 128 + ((4 * s2 + g) ^ sw(i)) * 16;
  {
    const int r0 = 8 * (g & 1) + qq;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) off2[c4] = r0 * 128 + ((2 * c4 + (p4 >> 1)) ^ sw(r0)) * 16 + 8 * (p4 & 1);
  }

  // -I as the B operand of iterate tile t: lane (i, g) holds k = 8g .. 8g + 7 of column n = i
  bf16x8 NEGI[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) NEGI[t][j] = (8 * g + j == 16 * t + i) ? (__bf16)(-1.0f) : (__bf16)(0.0f);

  auto step = [&](int u, uint8_t* slot, uint8_t* bslot, f32x4 (&pt)[QW][2][64]) __attribute__((always_inline)) {
    // ---- phase 1: P_w[rows 4g + r][iterate 16 t + i].  Fragment reads run AD k-steps ahead
    // of the MFMAs, each strip's after its wait
    constexpr int AD = MPA_LSQP4_AD;
    wait_strip((AD - 1) / 2);  // the strips of the first AD k-steps (and B, older)
#if MPA_LSQP4_VACC
    // every wave starts its chain with the B MFMA: wave 0 DMA'd B, and its accumulators start
    // at -B (A operand: lane (i, g) = row i, iterates 8g .. 8g + 7 of the half, one 16-B read of
    // the row-major slot, against -I: exact, one nonzero product per output added to 0); the
    // other waves read a zero slot, so their chains start at 0 with no separate initialisation
    f32x4 p1[2];
    {
      const bf16x8 bfr = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
          (w == 0 ? bslot : &bzero[w][0]) + i * (PH * 2) + 16 * g));
      p1[0] = mfma_v0(bfr, NEGI[0]);
      p1[1] = mfma_v0(bfr, NEGI[1]);
    }
#else
    f32x4 p1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    if (w == 0) {
      // wave 0 DMA'd B: its accumulators start at -B, by one MFMA per iterate tile of the B rows
      // (A operand: lane (i, g) = row i, iterates 8g .. 8g + 7 of the half, one 16-B read of the
      // row-major slot) against -I (exact: one nonzero product per output, added to 0)
      const bf16x8 bfr = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(bslot + i * (PH * 2) + 16 * g));
      p1[0] = mfma(bfr, NEGI[0], p1[0]);
      p1[1] = mfma(bfr, NEGI[1], p1[1]);
    }
#endif
    {
    bf16x8 af[AD];
    auto rd1 = [&](int s) __attribute__((always_inline)) {
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(slot + off1[s & 1] + 2048 * (s >> 1)));
    };
#pragma unroll
    for (int s = 0; s < AD; ++s) af[s] = rd1(s);
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      __builtin_amdgcn_sched_barrier(0);
      if (s + AD < NKS && ((s + AD) & 1) == 0) wait_strip((s + AD) / 2);
#if MPA_LSQP4_PROBE & 4
      (void)af;
#elif MPA_LSQP4_VACC
      mfma_v(p1[0], af[s % AD], XF[s][0]);
      mfma_v(p1[1], af[s % AD], XF[s][1]);
#else
      p1[0] = mfma(af[s % AD], XF[s][0], p1[0]);
      p1[1] = mfma(af[s % AD], XF[s][1], p1[1]);
#endif
      if (s + AD < NKS) af[s % AD] = rd1(s + AD);
    }
    __builtin_amdgcn_sched_barrier(0);
#if MPA_LSQP4_VACC
    mfma_v_settle(p1[0], p1[1]);
#endif
    }
    // phase 2's column tiles in chunks of 4 = one strip (8 transposed reads), double-buffered:
    // the reads of chunk c + 1 are issued before the MFMAs of chunk c; chunk 0's go out before
    // the reduce's barrier (they read only this wave's slot)
    constexpr int CH = 4;
    constexpr int P2L = MPA_LSQP4_P2L;  // chunks of reads in flight ahead of the MFMAs
    s16x4 tb[P2L + 1][CH][2];
    auto rd = [&](int c, s16x4 (&d)[CH][2]) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < CH; ++k) {
#if MPA_LSQP4_PROBE & 8  // timing probe 8: half the phase-2 reads (odd tiles reuse the even tile's)
        if (k & 1) {
          d[k][0] = d[k - 1][0];
          d[k][1] = d[k - 1][1];
          continue;
        }
#endif
        const uint8_t* src = slot + off2[k] + 2048 * c;
        d[k][0] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src));
        d[k][1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src + 4 * 128));
      }
    };
    rd(0, tb[0]);
    // ---- reduce, one barrier: every wave sums the four partials (wave order; wave 0's carry
    // -B) into R in the accumulator layout (rows 4g + r, iterate 16t + i), splits it into bf16
    // hi + lo, and moves the halves into phase 2's A operand with two lane swaps:
    //   RF[t] lane (i, g) = k 8g .. 8g + 7 = hi rows 0-7 | hi 8-15 | lo 0-7 | lo 8-15 (g = 0..3)
    // from lane groups' (H_g, L_g) = rows 4g .. 4g + 3: permlane32 (H, L) -> X = (H0 H1 L0 L1),
    // Y = (H2 H3 L2 L3); permlane16 (X, Y) -> X = (H0 H2 L0 L2), Y = (H1 H3 L1 L3) = the first
    // and second four k of every lane group
    bf16x8 RF[2];
#if MPA_LSQP4_PROBE & 2
    if (true) {  // timing probe: no cross-wave exchange (own partial only, no barrier)
      f32x4 pv[2][QW];
      for (int t = 0; t < 2; ++t)
        for (int ww = 0; ww < QW; ++ww) pv[t][ww] = p1[t];
#else
    pt[w][0][lane] = p1[0];
    pt[w][1][lane] = p1[1];
    barrier();
    {
#endif
      const int64_t row0 = int64_t(kb0 + u) * PRB + 4 * g;
      const bool ragged = !FULL && int64_t(kb0 + u + 1) * PRB > rows;  // wave-uniform
#if !(MPA_LSQP4_PROBE & 2)
      f32x4 pv[2][QW];  // all eight reads in flight at once
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ww = 0; ww < QW; ++ww) pv[t][ww] = pt[ww][t][lane];
#endif
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 v = pv[t][0];
#pragma unroll
        for (int ww = 1; ww < QW; ++ww) v += pv[t][ww];
        if (ragged) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = row0 + r < rows ? v[r] : 0.f;  // rows past the end: R = 0
        }
        uint32_t H[2], L[2];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          // packed conversions (v_cvt_pk_bf16_f32, round to nearest even): hi of two rows at
          // once, back to fp32 by a shift / mask, lo of the remainders at once
          H[d] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{v[2 * d], v[2 * d + 1]}, bf16x2));
          const float h0 = __uint_as_float(H[d] << 16), h1 = __uint_as_float(H[d] & 0xffff0000u);
          L[d] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{v[2 * d] - h0, v[2 * d + 1] - h1}, bf16x2));
        }
        uint32_t X[2], Y[2];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto sa = __builtin_amdgcn_permlane32_swap(H[d], L[d], false, false);
          const auto sb = __builtin_amdgcn_permlane16_swap(sa[0], sa[1], false, false);
          X[d] = sb[0];
          Y[d] = sb[1];
        }
        RF[t] = __builtin_bit_cast(bf16x8, make_uint4(X[0], X[1], Y[0], Y[1]));
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // chunk 1's reads stay behind the reduce (registers)
    // ---- phase 2: G_w^T[it][col] += sum_k R-image[it][k] A[row(k)][col]; strip c of the slot
    // is refilled with block u + 2's once chunk c's MFMAs have consumed its reads
    dma_b(kb0 + u + 2, bslot);
    const Blk nb2 = blk(kb0 + u + 2);
    uint32_t vf[2] = {vfull[0], vfull[1]}, vp[2] = {vpart[0], vpart[1]};
    if (!FULL && nb2.nv < PRB) voffs(nb2.nv, vf, vp);
#pragma unroll
    for (int c = 0; c < NCT / CH; ++c) {
#if MPA_LSQP4_P2I
      // the reads of chunk c + 1 go out BETWEEN this chunk's MFMAs, one per MFMA gap, instead of
      // as a cluster of eight before them (one wave per SIMD: clustered issue stretches the gaps)
      static_assert(P2L == 1, "interleaved phase-2 reads look one chunk ahead");
      lgkm_wait<0>();  // this chunk's reads, issued during the previous chunk's MFMAs
      __builtin_amdgcn_sched_barrier(0);
      if (c + 1 < NCT / CH) rd(c + 1, tb[(c + 1) & 1]);
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const bf16x8 bt = __builtin_bit_cast(
            bf16x8, __builtin_shufflevector(tb[c & 1][k][0], tb[c & 1][k][1], 0, 1, 2, 3, 4, 5, 6, 7));
        G[0][CH * c + k] = mfma(RF[0], bt, G[0][CH * c + k]);
        G[1][CH * c + k] = mfma(RF[1], bt, G[1][CH * c + k]);
      }
      if (c + 1 < NCT / CH) {
#pragma unroll
        for (int j = 0; j < 2 * CH; ++j) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one LDS read
        }
      }
#else
      if (c == 0) {
#pragma unroll
        for (int c2 = 1; c2 < P2L; ++c2) rd(c2, tb[c2]);
      }
      if (c + P2L < NCT / CH) rd(c + P2L, tb[(c + P2L) % (P2L + 1)]);
      // one wait for this chunk's reads (the younger chunks' 8 P2L reads stay in flight)
      // instead of one per MFMA pair
      if (c + P2L < NCT / CH) lgkm_wait<2 * CH * P2L>();
      else lgkm_wait<0>();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const bf16x8 bt = __builtin_bit_cast(
            bf16x8, __builtin_shufflevector(tb[c % (P2L + 1)][k][0], tb[c % (P2L + 1)][k][1], 0, 1, 2, 3, 4, 5, 6, 7));
        G[0][CH * c + k] = mfma(RF[0], bt, G[0][CH * c + k]);
        G[1][CH * c + k] = mfma(RF[1], bt, G[1][CH * c + k]);
      }
#endif
      __builtin_amdgcn_sched_barrier(0);
#if !(MPA_LSQP4_PROBE & 1)  // timing probe 1: no strip DMAs in the loop (A stays stale in LDS)
      dma_strip(nb2, vf, vp, c, slot);
#endif
    }
#if !(MPA_LSQP4_PROBE & 16)  // timing probe 16: no L2 prefetch in the loop
    pf(kb0 + u + 2 + pfd);
#endif
  };
#if MPA_MEASURE
  unsigned long long clk0 = 0, rt0 = 0;
  if (tid == 0) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
#endif
  for (int u = 0; u < nb; u += 2) {
    step(u, my0, bring[0], part[0]);
    if (u + 1 < nb) step(u + 1, my1, bring[1], part[1]);
  }
#if MPA_MEASURE
  if (tid == 0 && bx < kClockSlots && batch.ntasks >= 2) {
    const unsigned long long clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    g_lsqp4_clk[bx][0] = clk0;
    g_lsqp4_clk[bx][1] = rt0;
    g_lsqp4_clk[bx][2] = clk1;
    g_lsqp4_clk[bx][3] = rt1;
    g_lsqp4_clk[bx][4] = (unsigned long long)nb;
  }
#endif
#undef MPA_VMCNT
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
  bool cx = false;
  if (ng == 1) {
    cx = disarmed(a.go, a.seq);
    if (!cx)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) store_out(t, ct, G[t][ct]);
  } else {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) st_wt(slab + size_t(q) * qstride + (t * NCT + ct) * 64 + lane, G[t][ct]);
    if (batch.xred) return;  // lsqp4_reduce_kernel sums the partials, writes G and publishes
    unsigned idx = unsigned(q), count = unsigned(ng), stride = 1;
    int lvl_off = 0, lvl_cap = (kLsqpMaxGroups + PF - 1) / PF;
    for (;;) {
#if MPA_LSQP4_PROBE & 32
      break;
#endif
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
      if (next == 1) cx = disarmed(a.go, a.seq);
      const f32x4* src = slab + size_t(first) * stride * qstride;
      // JB tiles x PF members of loads in flight at once (clamped to member 0 past the group,
      // their sums selected away): one wave reduces its 64 KiB slice of the group, and with
      // one load chain per tile (each member's load waited for before the next issued) a
      // single-task launch spent ~0.2 ms in its four tree levels (c5n8, profiles/r06_pergpu.txt).
      // Summed in member order as before, so the result is bitwise the same.
#pragma unroll 1
      for (int jb = 0; jb < 2 * NCT; jb += kTreeJB) {
        f32x4 v[PF][kTreeJB];
#pragma unroll
        for (int m = 0; m < PF; ++m) {
          const size_t mo = size_t(unsigned(m) < gsize ? m : 0) * stride * qstride;
#pragma unroll
          for (int jj = 0; jj < kTreeJB; ++jj) v[m][jj] = ld_wt(src + mo + (jb + jj) * 64 + lane);
        }
#pragma unroll
        for (int jj = 0; jj < kTreeJB; ++jj) {
          f32x4 s = v[0][jj];
#pragma unroll
          for (int m = 1; m < PF; ++m) {
            const f32x4 t = s + v[m][jj];
            if (unsigned(m) < gsize) s = t;
          }
          const int j2 = jb + jj;
          if (next == 1) {
            if (!cx) store_out(j2 / NCT, j2 % NCT, s);
          } else {
            st_wt(slab + size_t(first) * stride * qstride + j2 * 64 + lane, s);
          }
        }
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
      if (!cx) {  // every slice read the same go word
        publish_task(a.flag, a.seq, a.pub_local);
        publish_peer(a.flag2, a.seq);
      }
    }
  }
}

// ---- G over the row groups as a second launch, for a launch of ONE task (round 6, the default;
// MPA_LSQP4_XRED=0 keeps the in-kernel tree above).  In the tree the last arriver of a group sums
// it, so at the upper levels a handful of waves move 256 KiB each while the rest of the chip idles:
// a lone task's four levels took 105 us of its 1.04 ms launch (c5n8: the node's per-GPU launch at
// N = 8, and every lone stale re-dispatch; profiles/r06_c5_xred.txt).  A launch of several tasks
// keeps the tree: there each task completes on its own, as soon as its tree is summed, where a
// second launch would hold every task's completion until the slowest task's row groups finish
// (the native k-of-n loop's c5 case: the small local worker's latency 0.1 -> 1.8 ms).  Here every (task, half,
// wave) slice is split over 16 workgroups, one thread per 16-B element of G, and each thread sums
// that element's partials over the row groups in the tree's own order -- groups of PF in member
// order, level by level, the short last group of a level passed up as it is -- with a stack of
// one pending sum per level, so G is bitwise what the tree gives.  The task's last workgroup
// publishes.
constexpr int kRedThreads = 256;
constexpr int kRedChunks = (2 * NCT * 64) / kRedThreads;  // workgroups per (half, wave) slice
constexpr int kRedPerTask = 2 * QW * kRedChunks;           // workgroups per task
constexpr int kRedLevels = 6;                              // PF^5 >= kLsqpMaxGroups
constexpr int kRedBatch = 16;                              // partial loads in flight per thread
static_assert(kRedChunks * kRedThreads == 2 * NCT * 64, "whole slices");
static_assert(PF * PF * PF * PF * PF >= kLsqpMaxGroups, "levels");

__global__ void __launch_bounds__(kRedThreads) lsqp4_reduce_kernel(LsqpBatch batch) {
  const int ti = int(blockIdx.x) / kRedPerTask;
  if (ti >= batch.ntasks) return;
  const LsqpTask& a = batch.t[ti];
  const int ng = batch.grp0[ti + 1] - batch.grp0[ti];
  if (ng <= 1) return;  // lsqp4 stored and published that task itself
  const int r = int(blockIdx.x) % kRedPerTask;
  const int h = r / (QW * kRedChunks), w = (r / kRedChunks) % QW, chunk = r % kRedChunks;
  const int e = chunk * kRedThreads + int(threadIdx.x);  // element of the slice: tile j, lane
  const int j = e >> 6, lane = e & 63, t = j / NCT, ct = j % NCT, i = lane & 15, g = lane >> 4;
  const int cols = a.cols, c0 = w * QKW;
  const int nks = cols > c0 ? ((cols - c0) < QKW ? (cols - c0) : QKW) / 32 : 0;
  const int col = c0 + 16 * ct + i;
  const bool valid = ct < 2 * nks && col < cols;
  __shared__ int s_cx;
  if (threadIdx.x < 64) {  // one wave: the go word (host memory) and, in-kernel armed, a timed-out wait
    bool cx = disarmed(a.go, a.seq);
    if (a.door && (__hip_atomic_load(batch.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & 64u)) cx = true;
    if (threadIdx.x == 0) s_cx = cx;
  }
  if (valid) {
    const size_t wslab = size_t(2 * NCT) * 64, qstride = size_t(QW) * wslab;
    const f32x4* __restrict__ src =
        static_cast<const f32x4*>(a.slab) + (size_t(h) * kLsqpMaxGroups * QW + w) * wslab + e;
    f32x4 lv[kRedLevels];
    int n[kRedLevels];  // members summed at each level (the same in every thread)
#pragma unroll
    for (int l = 0; l < kRedLevels; ++l) n[l] = 0;
    // add x as the next member at level l0; a group of PF members goes up as one
    auto push = [&](int l0, f32x4 x) __attribute__((always_inline)) {
#pragma unroll
      for (int l = 0; l < kRedLevels; ++l) {
        if (l < l0) continue;
        if (n[l] == 0) lv[l] = x;
        else lv[l] = lv[l] + x;
        if (++n[l] < PF) return;
        n[l] = 0;
        x = lv[l];
      }
    };
    for (int q0 = 0; q0 < ng; q0 += kRedBatch) {
      f32x4 v[kRedBatch];
#pragma unroll
      for (int k = 0; k < kRedBatch; ++k) v[k] = ld_wt(src + size_t(q0 + k < ng ? q0 + k : q0) * qstride);
#pragma unroll
      for (int k = 0; k < kRedBatch; ++k)
        if (q0 + k < ng) push(0, v[k]);
    }
    // the short last group of each level goes up as the last member of the next; the lowest
    // level with members and none above is the root
    f32x4 res = lv[0];
    bool done = false;
#pragma unroll
    for (int l = 0; l < kRedLevels; ++l) {
      bool above = false;
#pragma unroll
      for (int m = l + 1; m < kRedLevels; ++m) above = above || n[m] > 0;
      if (!done && n[l] > 0) {
        if (above) {
          n[l] = 0;
          push(l + 1, lv[l]);
        } else {
          res = lv[l];
          done = true;
        }
      }
    }
    __syncthreads();  // s_cx
    if (!s_cx) *reinterpret_cast<f32x4*>(static_cast<float*>(a.out) + size_t(col) * K + PH * h + 16 * t + 4 * g) = res;
  } else {
    __syncthreads();
  }
  drain_vm();
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    uint32_t* c = &a.ctr[2 * 8 * kLsqpCtrPerSlice];  // the slice-completion counter the tree path uses
    const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == unsigned(kRedPerTask)) {
      __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (!s_cx) {
        publish_task(a.flag, a.seq, a.pub_local);
        publish_peer(a.flag2, a.seq);
      }
    }
  }
}

static bool xred_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("MPA_LSQP4_XRED");
    return !(e && *e == '0');
  }();
  return on;
}

}  // namespace

#if MPA_MEASURE
void lsqp4_clock_dump() {
  static unsigned long long h[kClockSlots][5];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_lsqp4_clk), sizeof(h)) != hipSuccess) return;
  std::vector<double> ghz, us, cyc;
  for (int b = 0; b < kClockSlots; ++b)
    if (h[b][3] > h[b][1] && h[b][2] > h[b][0] && h[b][4] > 0) {
      ghz.push_back(double(h[b][2] - h[b][0]) / double(h[b][3] - h[b][1]) * 0.1);  // 100 MHz realtime
      us.push_back(double(h[b][3] - h[b][1]) / 100.0);
      cyc.push_back(double(h[b][2] - h[b][0]) / double(h[b][4]));
    }
  if (ghz.empty()) return;
  std::sort(ghz.begin(), ghz.end());
  std::sort(us.begin(), us.end());
  std::sort(cyc.begin(), cyc.end());
  std::fprintf(stderr, "lsqp4 clock: %zu workgroups of the last multi-task launch, in-kernel clock median %.3f GHz "
               "(min %.3f, max %.3f), block loop median %.1f us, %.0f shader cycles per 16-row block (median)\n",
               ghz.size(), ghz[ghz.size() / 2], ghz.front(), ghz.back(), us[us.size() / 2], cyc[cyc.size() / 2]);
}
#endif

hipError_t launch_lsqp4(const LsqpBatch& a0, hipStream_t s) {
  const int pairs = a0.grp0[a0.ntasks];
  if (pairs <= 0) return hipErrorInvalidValue;
  const int grid = (pairs + 7) / 8 * 16;
  LsqpBatch a = a0;
  bool full = true, multi = false;
  for (int t = 0; t < a.ntasks; ++t) {
    full = full && a.t[t].cols == kLsqpMaxCols && a.t[t].rows % PRB == 0;
    multi = multi || a.grp0[t + 1] - a.grp0[t] > 1;
    if (a.grp0[t + 1] - a.grp0[t] > kLsqpMaxGroups) return hipErrorInvalidValue;
  }
  a.xred = xred_enabled() && multi && a.ntasks == 1;
  const bool armed = batch_armed(a);
  if (armed && full) hipLaunchKernelGGL((lsqp4_kernel<true, true>), dim3(grid), dim3(QT), 0, s, a);
  else if (armed) hipLaunchKernelGGL((lsqp4_kernel<true, false>), dim3(grid), dim3(QT), 0, s, a);
  else if (full) hipLaunchKernelGGL((lsqp4_kernel<false, true>), dim3(grid), dim3(QT), 0, s, a);
  else hipLaunchKernelGGL((lsqp4_kernel<false, false>), dim3(grid), dim3(QT), 0, s, a);
  if (a.xred) hipLaunchKernelGGL(lsqp4_reduce_kernel, dim3(a.ntasks * kRedPerTask), dim3(kRedThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace mpa
