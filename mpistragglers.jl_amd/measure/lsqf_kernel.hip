// Single-pass batched least squares (BASELINE configs[4], "c5"):
//     G_i = A_i^T (A_i X - B_i)      A_i rows x cols bf16, X cols x 64 bf16, B_i rows x 64 bf16
// with A read from HBM ONCE.  The two-pass kernels (lsqb_kernel.hip) read A twice because
// the fp32 accumulator of G (cols x 64 x 4 B = 512 KiB at 2048 columns) is a whole CU's
// register file.  Here the columns are split over a GROUP of P workgroups (P = ceil(cols /
// 512), one per CU), each holding G for its 512-column slice in registers, and the group
// exchanges, per block of 16 rows, the partial residuals of its slices:
//
//   phase 1   member p: R_p = A[rows, slice p] X[slice p, :]      (16 x 64 fp32, MFMA)
//   exchange  R_p -> global memory (write-through stores, then a flag tagged (seq, block))
//   residual  R = sum_p R_p (member order) - B                     (bf16 hi + lo)
//   phase 2   G[slice p] += A[rows, slice p]^T R                    (MFMA; A^T by
//             transposed LDS reads of the same block)
//
// Workgroup = 8 compute waves + 4 loader waves, 3 waves per SIMD (168 VGPRs each).  The
// loaders stream 16-row blocks of the member's slice HBM -> VGPR -> an 8-slot LDS ring,
// F_D blocks ahead (wave-specialised because vmcnt is in order per wave: a compute wave
// that waits on an exchange load would also wait on every A prefetch of its own).  Compute
// wave w: phase 1 on iterate tile n = w & 3 over half kh = w >> 2 of the slice's columns
// (X half-slice resident, 32 VGPRs), the two halves added in LDS in kh order; phase 2 on
// columns 64 w .. 64 w + 63 (G: 64 VGPRs).  The residual of block t - F_LAG is formed at
// block t, so the partners' partials have F_LAG blocks of time to arrive.  Ring slots,
// pair partials and the residual image are handed over by LDS counters.
//
// Groups form dynamically (a ticket taken at start), so a group only waits for workgroups
// that are already running; every wait is bounded (spin_ticks).  The G slices of all groups
// are summed in group order by the last group to finish the slice (deterministic), and the
// task's last slice publishes completion.
//
// MFMA maps (cdna_hip_programming.md §3): 16x16x32 bf16 A[m=i][k=8g+j], B[k=8g+j][n=i];
// 16x16x16 bf16 A[m=i][k=4g+j], B[k=4g+j][n=i]; C/D[m=4g+r][n=i]; lane l: i = l&15, g = l>>4.
#include <hip/hip_runtime.h>

#include <cstdio>

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

constexpr int K = kLsqbIterates;          // 64
constexpr int F_CW = 8;                   // compute waves
constexpr int F_THREADS = (F_CW + 4) * 64;  // + 4 loader waves
constexpr int F_RB = 16;                  // rows per block
constexpr int F_W = kLsqfSlice;           // 512 columns per member
constexpr int F_NB = 6;                   // LDS ring slots
constexpr int F_LAG = 4;                  // residual of block t - F_LAG is formed at block t
constexpr int F_D = 3;                    // loader: blocks in flight beyond the one stored
constexpr int F_AS = F_W * 2 + 16;        // LDS bytes per A row in a slot (padded)
constexpr int F_BRS = K * 2 + 16;         // LDS bytes per B row in a slot (padded)
constexpr int F_SLOT = F_RB * F_AS + F_RB * F_BRS;  // A then B rows of a block: 18,944 B
constexpr int F_RS = 80;                  // residual image: per iterate hi rows 0-15, lo rows 0-15, pad
constexpr int F_RES = K * F_RS;           // one image (5 KiB)
constexpr int F_NR = 3;                   // residual images in the LDS ring
constexpr int F_PAIR = 4 * 64 * 16;       // kh = 1 phase-1 partials of one block (4 KiB)
constexpr int F_XST = 4 * kLsqfMaxP * 1024;  // members' partials of one block, landed by DMA
// LDS counters: full[NB], free[NB], pub[8], put[4], get[4], res, res_free
constexpr int F_NCNT = 2 * F_NB + 8 + 4 + 4 + 2;
static_assert(kLsqfXR >= 2 * F_LAG + 1, "exchange ring must outlive the slowest reader");

__device__ __forceinline__ f32x4 mfma32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ uint16_t bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return uint16_t((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_f32(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

__device__ __forceinline__ unsigned lds_load(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_inc(unsigned* p) {
  __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// this wave waits until an LDS counter reaches `want`; false on timeout (error flagged)
// MPA_LSQF_DBG=16 + mode: shader cycles spent per wave role in each wait, summed over launches
// ([role: loader, kh0, kh1][full, get, put, res, exchange, free, loop, blocks])
__device__ unsigned long long g_lsqf_prof[3][12];
struct Prof {
  bool on;
  unsigned long long c[12];
};
__device__ __forceinline__ unsigned long long now_cyc() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ bool lds_wait(const unsigned* p, unsigned want, unsigned long long t0,
                                         unsigned long long ticks, unsigned* err, Prof& pf, int k) {
  const unsigned long long c0 = pf.on ? now_cyc() : 0;
  struct Add {
    Prof& pf; int k; unsigned long long c0;
    __device__ ~Add() { if (pf.on) pf.c[k] += now_cyc() - c0; }
  } add_{pf, k, c0};
  // the clock (a scalar memory read) only every 256 polls: it sat on every handover's path
  for (unsigned k = 1; int(lds_load(p) - want) < 0; ++k) {
    __builtin_amdgcn_s_sleep(1);
    if ((k & 255) == 0 && rt_now() - t0 > ticks) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
  return true;
}
__device__ __forceinline__ void lgkm_drain() { __builtin_amdgcn_s_waitcnt(0xc07f); }  // lgkmcnt(0)

// (tag << 32 | count) word: count + 1, restarting at 1 under a new tag; the count before
__device__ unsigned tagged_inc(unsigned long long* w, unsigned tag) {
  unsigned long long old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    const bool cur = unsigned(old >> 32) == tag;
    const unsigned long long nv = cur ? old + 1 : ((unsigned long long)tag << 32) | 1ull;
    if (__hip_atomic_compare_exchange_strong(w, &old, nv, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      return cur ? unsigned(old) : 0u;
  }
}
__device__ unsigned tagged_count(unsigned long long* w, unsigned tag) {
  const unsigned long long v = __hip_atomic_fetch_add(w, 0ull, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  return unsigned(v >> 32) == tag ? unsigned(v) : 0u;
}

// Group formation (one lane per workgroup).  The partial residuals of a group whose members
// share an XCD go through that XCD's L2 (plain stores, L1-bypassing loads); a group spread
// over XCDs needs write-through stores, which drop the line from L2, so its hand-offs run at
// the cross-XCD latency.  A workgroup takes a ticket on its XCD (HW_REG_XCC_ID) and counts
// itself in; once the whole grid has (every workgroup of the launch is running or has run
// this far, so the wait cannot deadlock), each XCD's first P * floor(n_x / P) workgroups form
// same-XCD groups and the remainders, taken XCD by XCD, form mixed ones.  Placement decides
// only speed: every workgroup computes the same census.
__device__ void form_group(const LsqfBatch& b, int P, int& grp, int& mp, int& mixed) {
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  xcc &= 7;
  const unsigned tx = tagged_inc(&b.tick[xcc], b.tag);
  tagged_inc(&b.tick[8], b.tag);
  const unsigned grid = gridDim.x;
  const unsigned long long t0 = rt_now();
  unsigned k = 1;
  while (tagged_count(&b.tick[8], b.tag) < grid) {
    __builtin_amdgcn_s_sleep(4);
    if ((++k & 15) == 0 && rt_now() - t0 > b.spin_ticks) {
      __hip_atomic_fetch_or(b.err, 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      grp = -1;
      return;
    }
  }
  int before = 0, full_all = 0, left_before = 0, full_x = 0;
  for (unsigned y = 0; y < 8; ++y) {
    const int c = int(tagged_count(&b.tick[y], b.tag));
    const int f = (b.dbg & 15) == 7 ? 0 : c / P;  // probe: every group mixed
    full_all += f;
    if (y < xcc) {
      before += f;
      left_before += c - f * P;
    }
    if (y == xcc) full_x = f;
  }
  if (int(tx) < full_x * P) {
    grp = before + int(tx) / P;
    mp = int(tx) % P;
    mixed = 0;
  } else {
    const int L = left_before + int(tx) - full_x * P;
    grp = full_all + L / P;
    mp = L % P;
    mixed = 1;
  }
}

__global__ void __launch_bounds__(F_THREADS) lsqf_kernel(LsqfBatch batch) {
  extern __shared__ __attribute__((aligned(16))) uint8_t f_lds[];
  uint8_t* ring = f_lds;                        // F_NB slots
  uint8_t* res = ring + F_NB * F_SLOT;          // [F_NR] residual images
  uint8_t* pairbuf = res + F_NR * F_RES;        // [2][4 tiles][64 lanes] f32x4
  uint8_t* xst = pairbuf + 2 * F_PAIR;          // [4 tiles][members][64 lanes] f32x4
  unsigned* cnt = reinterpret_cast<unsigned*>(xst + F_XST);
  unsigned* full_cnt = cnt;
  unsigned* free_cnt = cnt + F_NB;
  unsigned* pub_cnt = cnt + 2 * F_NB;   // per block t % 8
  unsigned* put_cnt = cnt + 2 * F_NB + 8;
  unsigned* get_cnt = put_cnt + 4;
  unsigned* res_cnt = get_cnt + 4;
  unsigned* res_free = res_cnt + 1;
  __shared__ int s_grp, s_p, s_mixed;
  __shared__ unsigned s_last;

  const int tid = threadIdx.x, lane = tid & 63, i = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // a cancelled pre-armed launch returns before taking a ticket (every workgroup alike)
  if (batch.ntasks > 0 && disarmed(batch.t[0].go, batch.t[0].seq)) return;
  if (tid < F_NCNT) cnt[tid] = 0;
  const int P = batch.P;
  if (tid == 0) form_group(batch, P, s_grp, s_p, s_mixed);
  __syncthreads();
  const int G_all = s_grp, p = s_p;
  const bool mixed = s_mixed != 0;
  if (G_all < 0) return;  // group formation timed out (error flagged)
  int ti = 0;
  while (ti + 1 < batch.ntasks && G_all >= batch.grp0[ti + 1]) ++ti;
  const LsqfTask& a = batch.t[ti];
  const int grp = G_all - batch.grp0[ti];
  const int ngroups = batch.grp0[ti + 1] - batch.grp0[ti];
  const int64_t rows = a.rows;
  const int cols = a.cols;
  const int64_t nblocks = (rows + F_RB - 1) / F_RB;
  int nb = nblocks > grp ? int((nblocks - grp + ngroups - 1) / ngroups) : 0;  // this group's blocks
  const int c0 = p * F_W;
  const unsigned long long ticks = batch.spin_ticks;
  const unsigned long long t0 = rt_now();
  const int mode = batch.dbg & 15;
  const int skip = mode == 4 ? (batch.dbg >> 8) : 0;  // probe: parts of the no-exchange skeleton left out
  Prof pf{(batch.dbg & 16) != 0, {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}};
  const unsigned long long c_start = pf.on ? now_cyc() : 0;
  // the group's exchange ring: [XR][P][4 tiles][64 lanes] f32x4 partials, flags [XR][P]
  float* xbuf = static_cast<float*>(a.xbuf) + size_t(grp) * kLsqfXR * P * (4 * 64 * 4);
  unsigned long long* xflag = a.xflag + size_t(grp) * kLsqfXR * P;

  if (wave >= F_CW) {
    // ---------------- loader waves: rows 4 lw .. 4 lw + 3 of every block ----------------
    const int lw = wave - F_CW;
    const uint16_t* __restrict__ A = static_cast<const uint16_t*>(a.A);
    const int col = c0 + 8 * lane < cols ? c0 + 8 * lane : 0;  // columns past cols: column 0
    const uint16_t* __restrict__ Bm = static_cast<const uint16_t*>(a.B);
    const int brow = 8 * (lw & 1) + (lane >> 3);  // B: waves 0, 1 rows 0-7, 8-15 (2, 3 re-read, unused)
    // s_waitcnt vmcnt(15) (expcnt, lgkmcnt unchecked): the three younger stages (five loads
    // each) stay in flight.  Written out because the compiler's own wait, placed after the
    // slot-free spin loop, fell back to vmcnt(4)
    constexpr int kVmcnt15 = 0xF | (0x7 << 4) | (0xF << 8);
    // four stages of four rows in named registers (F_D = 3 blocks in flight beyond the one
    // being stored); a struct passed to a helper by reference stayed in scratch memory
    static_assert(F_D == 3, "the loader pipeline below is written for three blocks ahead");
    const int64_t lda = a.lda;
    auto rowat = [&](int t, int q) __attribute__((always_inline)) -> int64_t {
      const int tc = t < nb ? t : (nb > 0 ? nb - 1 : 0);  // past the end: re-read, unused
      const int64_t r = (int64_t(grp) + int64_t(tc) * ngroups) * F_RB + q;
      return r < rows ? r : rows - 1;
    };
    auto rowp = [&](int t, int q) __attribute__((always_inline)) -> const uint4* {
      return reinterpret_cast<const uint4*>(A + rowat(t, 4 * lw + q) * lda + col);
    };
    auto browp = [&](int t) __attribute__((always_inline)) -> const uint4* {
      return reinterpret_cast<const uint4*>(Bm + rowat(t, brow) * K + 8 * (lane & 7));
    };
    bool ok = true;
    auto slot_free = [&](int t) __attribute__((always_inline)) -> uint8_t* {
      const int slot = t % F_NB;
      // the slot's previous block (t - F_NB) must be released by all compute waves
      ok = ok && lds_wait(&free_cnt[slot], unsigned(F_CW) * unsigned(t / F_NB), t0, ticks, batch.err, pf, 5);
      return ring + slot * F_SLOT;
    };
    auto slot_full = [&](int t) __attribute__((always_inline)) {
      lgkm_drain();
      if (lane == 0) lds_inc(&full_cnt[t % F_NB]);
    };
#define LSQF_ISSUE(x, t) \
  x##0 = *rowp(t, 0);    \
  x##1 = *rowp(t, 1);    \
  x##2 = *rowp(t, 2);    \
  x##3 = *rowp(t, 3);    \
  x##4 = *browp(t)
#define LSQF_STORE(x, t)                                                                  \
  __builtin_amdgcn_s_waitcnt(kVmcnt15); /* this stage's 5 loads */                        \
  if ((t) < nb && ok) {                                                                   \
    uint8_t* s_ = slot_free(t);                                                           \
    uint8_t* d_ = s_ + 4 * lw * F_AS + 16 * lane;                                         \
    *reinterpret_cast<uint4*>(d_) = x##0;                                                 \
    *reinterpret_cast<uint4*>(d_ + F_AS) = x##1;                                          \
    *reinterpret_cast<uint4*>(d_ + 2 * F_AS) = x##2;                                      \
    *reinterpret_cast<uint4*>(d_ + 3 * F_AS) = x##3;                                      \
    if (lw < 2) *reinterpret_cast<uint4*>(s_ + F_RB * F_AS + brow * F_BRS + 16 * (lane & 7)) = x##4; \
    slot_full(t);                                                                         \
  }
    uint4 sa0, sa1, sa2, sa3, sa4, sb0, sb1, sb2, sb3, sb4, sc0, sc1, sc2, sc3, sc4, sd0, sd1, sd2, sd3, sd4;
    LSQF_ISSUE(sa, 0);
    LSQF_ISSUE(sb, 1);
    LSQF_ISSUE(sc, 2);
    for (int t = 0; t < nb && ok; t += 4) {
      LSQF_ISSUE(sd, t + 3);
      LSQF_STORE(sa, t);
      LSQF_ISSUE(sa, t + 4);
      LSQF_STORE(sb, t + 1);
      LSQF_ISSUE(sb, t + 5);
      LSQF_STORE(sc, t + 2);
      LSQF_ISSUE(sc, t + 6);
      LSQF_STORE(sd, t + 3);
    }
#undef LSQF_ISSUE
#undef LSQF_STORE
  } else {
    // ---------------- compute waves ----------------
    const int cw = wave, n = cw & 3, kh = cw >> 2;
    const uint16_t* __restrict__ X = static_cast<const uint16_t*>(a.X);
    // phase-1 B operands: X[c0 + 256 kh + 32 s + 8 g + j][16 n + i]
    bf16x8 XF[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      s16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + 256 * kh + 32 * s + 8 * g + j;
        v[j] = c < cols ? short(X[size_t(c) * K + 16 * n + i]) : short(0);
      }
      XF[s] = __builtin_bit_cast(bf16x8, v);
    }
    f32x4 acc[4][4];  // [iterate tile][column tile] of G^T, columns 64 cw + 16 ct
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) acc[u][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned long long seqtag = (unsigned long long)a.seq << 32;
    const int q4 = (lane >> 2) & 3, p4 = lane & 3;
    // kh 0 waves publish the member's partial tiles (stores only), kh 1 waves gather the
    // members' partials and form the residual (loads only): vmcnt is in order per wave, so a
    // wave that did both would wait for its own write-through stores behind every load.
    //
    // kh 0: the flag of block t - 1 goes up after block t's stores are issued, once every
    // store but those two has completed (vmcnt(2)); the last block's at the end of phase 1.
    int pend = -1;
    auto raise_flag = [&](bool last) __attribute__((always_inline)) {
      if (pend < 0) return;
      if (last)
        drain_vm();
      else if (mixed)
        __builtin_amdgcn_s_waitcnt(0x2 | (0x7 << 4) | (0xF << 8));  // vmcnt(2): block t's two stores
      else
        __builtin_amdgcn_s_waitcnt(0x1 | (0x7 << 4) | (0xF << 8));  // vmcnt(1): block t's store
      if (lane == 0) {
        const unsigned old = __hip_atomic_fetch_add(&pub_cnt[pend & 7], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old == 4u * unsigned(pend >> 3) + 3u) {
          unsigned long long* f = &xflag[(pend % kLsqfXR) * P + p];
          if (mixed)
            __hip_atomic_store(f, seqtag | unsigned(pend + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else  // a plain store: the line stays in the group's L2
            __hip_atomic_store(f, seqtag | unsigned(pend + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      pend = -1;
    };
    // kh 1: block u's partials in flight one block ahead (loaded straight into LDS, no
    // registers held), block u + 1's flags two blocks ahead
    unsigned long long fl[kLsqfMaxP];
    uint8_t* xs = xst + n * (kLsqfMaxP * 1024);
    auto load_flags = [&](int b) __attribute__((always_inline)) {
      const unsigned long long* f = &xflag[(b % kLsqfXR) * P];
#pragma unroll
      for (int q = 0; q < kLsqfMaxP; ++q)  // members past P re-read member 0's flag
        fl[q] = __hip_atomic_load(&f[q < P ? q : 0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // block b's flags have all been seen up (polling again until they are), then its
    // partials are loaded: the loads follow the flags they depend on
    auto load_data = [&](int b) __attribute__((always_inline)) -> bool {
      const unsigned long long want = seqtag | unsigned(b + 1);
      const unsigned long long cx = pf.on ? now_cyc() : 0;
      bool good = true;
      if (mode >= 4 && mode != 7) return true;
      for (unsigned k = 1;; ++k) {
        bool all = true;
#pragma unroll
        for (int q = 0; q < kLsqfMaxP; ++q) all = all && fl[q] == want;
        if (all) break;
        __builtin_amdgcn_s_sleep(1);
        if ((k & 15) == 0 && rt_now() - t0 > ticks) {
          if (lane == 0) __hip_atomic_fetch_or(batch.err, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          good = false;
          break;
        }
        load_flags(b);
      }
      lgkm_drain();  // the previous block's reads of the landing area are done
#pragma unroll
      for (int q = 0; q < kLsqfMaxP; ++q)  // sc1 (aux 16): coherent with the other CUs' stores
        if (q < P)
          __builtin_amdgcn_global_load_lds(
              static_cast<const void*>(xbuf + ((size_t((b % kLsqfXR) * P + q) * 4 + n) * 64 + lane) * 4),
              (__attribute__((address_space(3))) void*)(xs + q * 1024), 16, 0, 16);
      if (pf.on) pf.c[4] += now_cyc() - cx;
      return good;
    };

    auto phase1 = [&](int t) __attribute__((always_inline)) -> bool {
      const int slot = t % F_NB;
      if (!lds_wait(&full_cnt[slot], 4u * unsigned(t / F_NB + 1), t0, ticks, batch.err, pf, 0)) return false;
      const unsigned long long c1 = pf.on ? now_cyc() : 0;
      const uint8_t* base = ring + slot * F_SLOT + i * F_AS + 2 * (256 * kh) + 16 * g;
      f32x4 r1 = f32x4{0.f, 0.f, 0.f, 0.f};
      if (mode != 8 && !(skip & 1)) {
#pragma unroll
        for (int s = 0; s < 8; ++s)
          r1 = mfma32(__builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + 64 * s)), XF[s], r1);
      }
      if (pf.on) {
        __builtin_amdgcn_sched_barrier(0);
        pf.c[9] += now_cyc() - c1;
      }
      f32x4* pb = reinterpret_cast<f32x4*>(pairbuf + (t & 1) * F_PAIR) + n * 64 + lane;
      if (kh == 1) {
        // hand the second half to wave n once it has taken block t - 2's out of this buffer
        if (!(skip & 8) && !lds_wait(&get_cnt[n], unsigned(t > 1 ? t - 1 : 0), t0, ticks, batch.err, pf, 1)) return false;
        *pb = r1;
        lgkm_drain();
        if (lane == 0) lds_inc(&put_cnt[n]);
        return true;
      }
      if (!(skip & 8) && !lds_wait(&put_cnt[n], unsigned(t + 1), t0, ticks, batch.err, pf, 2)) return false;
      r1 += *pb;  // kh 0 + kh 1, fixed order
      lgkm_drain();
      if (lane == 0) lds_inc(&get_cnt[n]);
      if (mode >= 4 && mode != 7) return true;  // probe: no exchange (G wrong)
      // publish the member's tile n (write-through)
      unsigned long long* d8 =
          reinterpret_cast<unsigned long long*>(xbuf + ((size_t((t % kLsqfXR) * P + p) * 4 + n) * 64 + lane) * 4);
      if (mixed) {
        const unsigned long long* s8 = reinterpret_cast<const unsigned long long*>(&r1);
        __hip_atomic_store(d8, s8[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d8 + 1, s8[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        *reinterpret_cast<f32x4*>(d8) = r1;
      }
      raise_flag(false);
      pend = t;
      return true;
    };

    auto phase2 = [&](int u) __attribute__((always_inline)) -> bool {
      // straight-line (a timeout flags the error and carries on): an early exit between the
      // updates of acc made the compiler keep two copies of the accumulators
      bool good = true;
      uint8_t* rbuf = res + (u % F_NR) * F_RES;
      const uint8_t* slot = ring + (u % F_NB) * F_SLOT;
      if (kh == 1) {
        // residual tile n (rows 4 g + r, iterate 16 n + i) = the members' partials in member
        // order - B; the buffer's previous image (block u - F_NR) released by every wave
        const unsigned long long cd = pf.on ? now_cyc() : 0;
        drain_vm();  // block u's partials (and block u + 1's flags) have landed
        if (pf.on) pf.c[8] += now_cyc() - cd;
        f32x4 v = *reinterpret_cast<const f32x4*>(xs + 16 * lane);
#pragma unroll
        for (int q = 1; q < kLsqfMaxP; ++q)
          if (q < P) v += *reinterpret_cast<const f32x4*>(xs + q * 1024 + 16 * lane);
        if (u + 1 < nb) {
          good = load_data(u + 1);
          if (u + 2 < nb && !(skip & 32)) load_flags(u + 2);
        }
        good = ((skip & 16) || lds_wait(res_free, unsigned(F_CW) * unsigned(u >= F_NR ? u - F_NR + 1 : 0), t0, ticks,
                                        batch.err, pf, 3)) && good;
        const int64_t rb = int64_t(grp) + int64_t(u) * ngroups;
        const int it = 16 * n + i;
        uint16_t hi[4], lo[4];
        if (mode != 5 && !(skip & 2)) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // B of the block came into the ring slot with A
          const uint16_t b = *reinterpret_cast<const uint16_t*>(slot + F_RB * F_AS + (4 * g + r) * F_BRS + 2 * it);
          const int64_t row = rb * F_RB + 4 * g + r;
          const float x = row < rows ? v[r] - bf16_f32(b) : 0.f;
          hi[r] = bf16_rne(x);
          lo[r] = bf16_rne(x - bf16_f32(hi[r]));
        }
        *reinterpret_cast<uint2*>(rbuf + it * F_RS + 8 * g) =
            make_uint2(uint32_t(hi[0]) | (uint32_t(hi[1]) << 16), uint32_t(hi[2]) | (uint32_t(hi[3]) << 16));
        *reinterpret_cast<uint2*>(rbuf + it * F_RS + 32 + 8 * g) =
            make_uint2(uint32_t(lo[0]) | (uint32_t(lo[1]) << 16), uint32_t(lo[2]) | (uint32_t(lo[3]) << 16));
        }
        lgkm_drain();
        if (lane == 0) lds_inc(res_cnt);
      }
      good = ((skip & 16) || lds_wait(res_cnt, 4u * unsigned(u + 1), t0, ticks, batch.err, pf, 3)) && good;
      const unsigned long long c2 = pf.on ? now_cyc() : 0;
      // phase 2: G^T[it][col] += res^T[it][row] A[row][col], one K = 32 MFMA per tile:
      // k 0-15 the hi residual of rows 0-15, k 16-31 the lo residual of the same rows
      const uint8_t* sb = slot + (8 * (g & 1) + q4) * F_AS + 2 * (64 * cw + 4 * p4);
      bf16x8 bt[4];
#pragma unroll
      for (int ct = 0; ct < 4 && !(skip & 4); ++ct) {
        // rows 8 (g & 1) + 4 h + q4, columns 64 cw + 16 ct + 4 p4: lane i gets column 16 ct + i
        const s16x4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sb + 32 * ct));
        const s16x4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sb + 4 * F_AS + 32 * ct));
        bt[ct] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int uu = 0; uu < 4 && mode != 6 && !(skip & 4); ++uu) {
        const bf16x8 ra = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(rbuf + (16 * uu + i) * F_RS + 16 * g));
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[uu][ct] = mfma32(ra, bt[ct], acc[uu][ct]);
      }
      lgkm_drain();
      if (pf.on) pf.c[10] += now_cyc() - c2;
      if (lane == 0) {
        lds_inc(&free_cnt[u % F_NB]);
        lds_inc(res_free);
      }
      return good;
    };

    // phase 1 runs F_LAG blocks ahead; phase 2 (the only writer of acc) runs once per
    // iteration of the second loop, so the accumulators stay in place
    bool ok = true;
    if (mode == 3) {  // probe: the loader alone (slots released unread)
      for (int u = 0; u < nb && ok; ++u) {
        ok = lds_wait(&full_cnt[u % F_NB], 4u * unsigned(u / F_NB + 1), t0, ticks, batch.err, pf, 0);
        if (lane == 0) lds_inc(&free_cnt[u % F_NB]);
      }
      nb = 0;
    }
    // lag >= 2: block b's flag goes up with phase 1 of b + 1, which must come before the
    // partials of b are gathered (phase 2 of b - 1, in the same iteration when lag is 2)
    const int lag = batch.lag >= 2 && batch.lag <= F_LAG ? batch.lag : F_LAG;
    for (int t = 0; t < lag && t < nb && ok; ++t) ok = phase1(t);
    if (kh == 0) {
      if (nb <= lag) raise_flag(true);
    } else if (nb > 0) {
      load_flags(0);
      ok = ok && load_data(0);
      if (nb > 1) load_flags(1);
    }
    for (int u = 0; u < nb && ok; ++u) {
      if (u + lag < nb) {
        ok = phase1(u + lag);
        if (kh == 0 && u + lag + 1 == nb) raise_flag(true);  // phase 1 is done
      }
      ok = ok && phase2(u);
    }
    // this wave's G columns of this group -> slab[grp][p][cw][u][ct][lane] f32x4
    float* part = static_cast<float*>(a.slab) + (size_t(grp) * P + p) * (F_CW * 16 * 64 * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        *reinterpret_cast<f32x4*>(part + (((cw * 4 + u) * 4 + ct) * 64 + lane) * 4) = acc[u][ct];
  }
  if (pf.on && lane == 0) {
    pf.c[6] = now_cyc() - c_start;
    pf.c[7] = unsigned(nb);
    const int role = wave >= F_CW ? 0 : 1 + (wave >> 2);
    for (int k = 0; k < 12; ++k) atomicAdd(&g_lsqf_prof[role][k], pf.c[k]);
  }
  drain_vm();
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old - a.sbase) == unsigned(ngroups - 1);
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      drain_vm();
    }
  }
  __syncthreads();
  if (!s_last) return;
  // the slice's last group: sum the groups' partials in group order, write G[col][iterate]
  constexpr int UNITS = F_CW * 16 * 64;  // f32x4 units per member partial
  const f32x4* base = reinterpret_cast<const f32x4*>(static_cast<const float*>(a.slab) + size_t(p) * (UNITS * 4));
  const size_t gstride = size_t(P) * UNITS;
  float* out = static_cast<float*>(a.out);
  for (int j = tid; j < UNITS; j += F_THREADS) {
    f32x4 s0 = base[j];
    for (int gq = 1; gq < ngroups; ++gq) s0 += base[size_t(gq) * gstride + j];
    // j = ((cw*4 + u)*4 + ct)*64 + l -> column c0 + 64 cw + 16 ct + (l & 15), iterates 16 u + 4 (l >> 4) + r
    const int l = j & 63, ct = (j >> 6) & 3, u = (j >> 8) & 3, cw = j >> 10;
    const int colo = c0 + 64 * cw + 16 * ct + (l & 15);
    if (colo < cols) *reinterpret_cast<f32x4*>(out + size_t(colo) * K + 16 * u + 4 * (l >> 4)) = s0;
  }
  drain_vm();
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[kLsqfMaxP], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old - a.tbase == unsigned(P - 1)) publish_done(a.flag, a.seq);
  }
}

}  // namespace

void lsqf_prof_dump() {
  unsigned long long h[3][12];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_lsqf_prof), sizeof(h)) != hipSuccess) return;
  static const char* role[3] = {"loader", "kh0", "kh1"};
  static const char* what[11] = {"full", "get", "put", "res", "exch", "free", "", "", "drain", "p1", "p2"};
  for (int r = 0; r < 3; ++r) {
    const double nbk = double(h[r][7] ? h[r][7] : 1);
    std::fprintf(stderr, "lsqf prof %-6s cycles/block: loop %.0f", role[r], double(h[r][6]) / nbk);
    for (int k = 0; k < 11; ++k)
      if (*what[k]) std::fprintf(stderr, "  %s %.0f", what[k], double(h[r][k]) / nbk);
    std::fprintf(stderr, "\n");
  }
}

size_t lsqf_lds_bytes() {
  return size_t(F_NB) * F_SLOT + F_NR * size_t(F_RES) + F_XST + 2 * size_t(F_PAIR) + sizeof(unsigned) * F_NCNT;
}

hipError_t launch_lsqf(const LsqfBatch& a, hipStream_t s) {
  const int grid = a.grp0[a.ntasks] * a.P;
  if (grid <= 0 || a.P < 1 || a.P > kLsqfMaxP) return hipErrorInvalidValue;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(lsqf_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lsqf_lds_bytes()));
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(lsqf_kernel, dim3(grid), dim3(F_THREADS), lsqf_lds_bytes(), s, a);
  return hipGetLastError();
}

}  // namespace mpa
