// lsq_grad_kernel: the worker compute of the BASELINE workload, g_i = A_i^T (A_i x - b_i),
// placed in the reference's compute slot (examples/iterative_example.jl:74 sleeps there).
//
// ONE pass over A (the single-pass requirement of SURVEY.md §7): a wave owns whole rows;
// lane l holds the 16-B vectors v*64 + l (v < VPL) of a row, so each load instruction of
// a wave reads 1 KiB contiguous; x and the running g stay in registers for the kernel.
//   per row:  dot = wave_sum(sum_v a_v . x_v);  r = dot - b[row];  g_v += r * a_v
// Rows are dealt to waves in tiles of RB rows, grid-strided so the grid sweeps one
// contiguous region of A at a time.
//
// Several workers posted by the same flush run as ONE launch (LsqBatch): workgroups
// [block0[t], block0[t+1]) serve task t.
//
// Cross-workgroup reduction, deterministic (no float atomics): the 4 waves of a
// workgroup add their g in LDS in wave order, the workgroup stores its partial into
// slab[block][:], and a fan-in-8 tree of arrival counters sums the partials in block
// order: the last arriver of each group of 8 carries the group's sum one level up, the
// last one writes the reply chunk and publishes completion.  Nothing waits on another
// workgroup, so the result never depends on how many workgroups are resident.
//
// Compile-time variants (MODE bits) exist for measurement (DESIGN.md §Kernel tuning; all of
// them are compiled only into the measurement build, make MEASURE=1):
//   M_CLAMP     branch-free loads: out-of-range rows/vectors read a clamped in-bounds
//               address and are multiplied by zero instead of branched around
//   M_DPP       wave reduction by DPP row ops + readlane instead of ds_bpermute
//   M_PREFETCH  register double buffer: the next tile's loads issue before this tile's math
//   M_NT        non-temporal loads of A (streamed once)
//   M_TREE_FENCE  reduction-tree hand-offs by plain stores + agent release / acquire fences
//               instead of write-through (sc1) stores and loads
//   M_BLOCKED   each workgroup streams ONE contiguous row range (its 1/grid of the task,
//               in whole tiles), its waves taking the range's tiles in turn, instead of
//               the grid sweeping the task's rows together
//   M_ARMED     (set per launch, not a tuning bit) every workgroup first waits on the task's
//               device doorbell (a device-armed task of a worker process, kernels.hpp)
//   M_HEAD      (set per launch) the fused head: workgroup 0 runs the epoch step first
//               (LsqBatch::head); a prologue the other launches must not carry (its mere
//               presence cost the c2 launch 19 %)
//   M_ROTATE    grid sweeps with the workgroup's tile rotated by one per sweep (below; c2's
//               shape, where it measured faster)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef MPA_MEASURE
#define MPA_MEASURE 0
#endif

#include "device_common.hpp"
#include "epoch_step.hpp"
#include "lsq_common.hpp"
#include "kernels.hpp"
#include "mpiasyncpools.h"

namespace mpa {
namespace {

using namespace dev;

enum : int { M_CLAMP = 1, M_DPP = 2, M_PREFETCH = 4, M_NT = 8, M_TREE_FENCE = 16, M_BLOCKED = 32, M_ARMED = 64, M_HEAD = 128,
             M_ROTATE = 256 };

template <typename T, int VPL, int RB, int MODE>
struct Tile {
  using P = Pack<T>;
  static constexpr int E = P::E;
  P d[RB][VPL];
  // the fused-head variants' b values, loaded with the tile (load_b): under the head's control
  // flow each row's b load was issued in its own branch and waited for there, one memory round
  // trip per row (c1's 16-row tiles: most of its tasks' time); clamped, they issue together,
  // before the token wait for a prefetched tile.  (fp32 kept its per-row loads in round 5: moving
  // them changed how the compiler contracted the row's update, r05bf; compute() now spells its
  // fused multiply-adds out, so the variants round alike whatever the loads' placement.)  Every
  // load() of a head tile is followed by its load_b(), the prefetching loop's included.
  static constexpr bool kHeadB = (MODE & M_HEAD) != 0;
  [[maybe_unused]] T bq[kHeadB ? RB : 1];

  // rows [base, base+RB): out-of-range rows/vectors either branch (default) or read a
  // clamped in-bounds address (M_CLAMP: the row's last valid row, vector 0 of the row for
  // lanes past cols) whose contribution is zeroed by x = 0 / res = 0
  __device__ __forceinline__ void load(const T* A, int64_t base, int64_t rows, int64_t lda, int lane,
                                       const bool (&vok)[VPL]) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int64_t r0 = base + rb;
      if constexpr (MODE & M_CLAMP) {
        const int64_t r = r0 < rows ? r0 : rows - 1;
        const P* row = reinterpret_cast<const P*>(A + r * lda);
#pragma unroll
        for (int v = 0; v < VPL; ++v) d[rb][v] = ld16<T, (MODE & M_NT) != 0>(row + (vok[v] ? v * 64 + lane : 0));
      } else {
        const P* row = reinterpret_cast<const P*>(A + r0 * lda);
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
          if (r0 < rows && vok[v]) {
            d[rb][v] = ld16<T, (MODE & M_NT) != 0>(row + v * 64 + lane);
          } else {
#pragma unroll
            for (int e = 0; e < E; ++e) d[rb][v].v[e] = T(0);
          }
        }
      }
    }
  }

  __device__ __forceinline__ void load_b(const T* __restrict__ bv, int64_t base, int64_t rows) {
    if constexpr (kHeadB) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int64_t r = base + rb;
        bq[rb] = bv[r < rows ? r : rows - 1];
      }
    }
  }

  // The row's dot and the g update are written as explicit fused multiply-adds in a fixed
  // order, so that every kernel variant (plain, head, armed, tail, pre-armed) rounds them the
  // same way whatever the surrounding code lets the compiler contract (moving
  // the fp32 head variant's b loads once changed its contraction by 1 ulp).
  static __device__ __forceinline__ T fmac(T a, T b, T c) {
    if constexpr (sizeof(T) == 8) return __builtin_fma(a, b, c);
    else return __builtin_fmaf(a, b, c);
  }

  __device__ __forceinline__ void compute(const T* __restrict__ bv, int64_t base, int64_t rows, const P (&xr)[VPL],
                                          P (&g)[VPL]) const {
    T dot[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      T s = T(0);
#pragma unroll
      for (int v = 0; v < VPL; ++v)
#pragma unroll
        for (int e = 0; e < E; ++e) s = fmac(d[rb][v].v[e], xr[v].v[e], s);
      dot[rb] = s;
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) dot[rb] = wave_sum<T, (MODE & M_DPP) != 0>(dot[rb]);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int64_t r = base + rb;
      T res;
      if constexpr (kHeadB) res = (r < rows) ? dot[rb] - bq[rb] : T(0);
      else res = (r < rows) ? dot[rb] - bv[r] : T(0);
#pragma unroll
      for (int v = 0; v < VPL; ++v)
#pragma unroll
        for (int e = 0; e < E; ++e) g[v].v[e] = fmac(res, d[rb][v].v[e], g[v].v[e]);
    }
  }
};

#if MPA_MEASURE
// measurement build (MPA_HEAD_STAMP=1 dumps them): s_memrealtime of a fused-head launch, by its head
// token: [0] workgroup 0 saw the go word, [1] it published the head token, [2] the first other
// workgroup saw the token, [3] the first task's last reducer began its sum, [4] the last publish,
// [5] workgroup 0 starts the step (after the acquire and its arguments), [6] the step's stores issued
constexpr int kHeadSlots = 4096;
__device__ unsigned long long g_head_stamp[kHeadSlots][7];
__device__ __forceinline__ void head_stamp(uint32_t token, int k, bool first) {
  unsigned long long* p = &g_head_stamp[token % kHeadSlots][k];
  if (first) atomicMin(p, rt_now());
  else atomicMax(p, rt_now());
}
#define MPA_HEAD_STAMP(tok, k, first) head_stamp(tok, k, first)
// measurement build (MPA_LSQ_STAMP=1 dumps them): s_memrealtime of the last launch, per workgroup
// [0] entry and [1] end of its block loop; the launch's last tree root start and last publish
constexpr int kLsqStampWgs = 1024;
__device__ unsigned long long g_lsq_wg[kLsqStampWgs][4];  // realtime entry / loop end, shader clock entry / loop end
__device__ unsigned g_lsq_xcc[kLsqStampWgs];             // the XCC the workgroup ran on (HW_REG_XCC_ID)
__device__ unsigned long long g_lsq_root, g_lsq_pub;
__device__ unsigned g_lsq_grid;
#define MPA_LSQ_WG_STAMP(k) \
  do {                     \
    if (threadIdx.x == 0 && blockIdx.x < kLsqStampWgs) {                                   \
      g_lsq_wg[blockIdx.x][k] = rt_now();                                                    \
      g_lsq_wg[blockIdx.x][2 + k] = __builtin_amdgcn_s_memtime();                            \
      if (k == 0) {                                                                          \
        unsigned xcc_;                                                                       \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                 \
        g_lsq_xcc[blockIdx.x] = xcc_ & 0xF;                                                  \
      }                                                                                      \
    }                                                                                        \
  } while (0)
#define MPA_LSQ_MAX_STAMP(v) atomicMax(&(v), rt_now())
#else
#define MPA_HEAD_STAMP(tok, k, first) (void)0
#define MPA_LSQ_WG_STAMP(k) (void)0
#define MPA_LSQ_MAX_STAMP(v) (void)0
#endif

template <typename T, int VPL, int RB, int MODE>
__global__ void __launch_bounds__(kThreads) lsq_grad_kernel(LsqBatch batch) {
  using P = Pack<T>;
  constexpr int E = P::E;
  __shared__ P red[VPL * 64];           // workgroup partial (VPL*64*E columns)
  __shared__ P red2[VPL == 1 ? 3 * 64 : 1];  // the one-level tree's partial sums 1-3
  __shared__ unsigned s_ticket, s_cancel;

  // which task of the batch this workgroup serves (wave-uniform scan over <= 16 entries)
  int ti = 0;
  while (ti + 1 < batch.ntasks && int(blockIdx.x) >= batch.block0[ti + 1]) ++ti;
  const LsqTask& a = batch.t[ti];
  const int blk = int(blockIdx.x) - batch.block0[ti];
  if constexpr ((MODE & M_ARMED) != 0)
    if (!wait_door(a.door, a.seq, batch.spin_ticks, batch.err)) return;  // device-armed
  MPA_LSQ_WG_STAMP(0);
#if MPA_MEASURE
  if (threadIdx.x == 0 && blockIdx.x == 0) g_lsq_grid = gridDim.x;
#endif
  // A pre-armed task its server cancelled (the host-memory go word holds its seq) computes
  // but neither writes its reply nor publishes.  The word is read ONCE, by the workgroup that
  // writes the reply, at that point: every lane of every workgroup reading it before any work
  // cost a 192-workgroup task ~125 us (profiles/r02_arm_go_word.txt).  Call with the whole
  // workgroup.
  auto cancelled = [&]() -> bool {
    if (!a.go) return false;
    if (threadIdx.x == 0)
      s_cancel = __hip_atomic_load(a.go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == a.seq;
    __syncthreads();
    return s_cancel != 0;
  };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const T* __restrict__ A = static_cast<const T*>(a.A);
  const T* __restrict__ bv = static_cast<const T*>(a.b);
  const T* __restrict__ xv = static_cast<const T*>(a.x);

  P xr[VPL], g[VPL];
  bool vok[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c0 = (v * 64 + lane) * E;
    vok[v] = c0 < a.cols;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if constexpr ((MODE & M_HEAD) == 0) xr[v].v[e] = (c0 + e < a.cols) ? xv[c0 + e] : T(0);
      g[v].v[e] = T(0);
    }
  }

  const int64_t rows = a.rows;
  int64_t step, base, hi;  // this wave's tiles: base, then nxt(), ... while < hi
  // Grid sweeps (not M_BLOCKED): sweep k covers rows [k step, (k + 1) step), one tile of
  // kWaves * RB rows per workgroup, workgroup blk taking tile blk of it -- or, M_ROTATE, tile
  // (blk + k) mod grid.  Motivated by a split by XCD (round-robin placement gives an XCD the
  // workgroups of one residue mod 8): the XCDs of one parity ended their loops ~12 us after the
  // other's in every c2 launch.  The split persists with the rotation (so it is not the tiles'
  // addresses), but c2 measured +0.4-1.2 % rotated in 7 of 7 same-box pairs; c3's 128-KiB tiles
  // -1.3 %, its delayed lone tasks -7 %, c1 level: only c2's shape rotates
  // (profiles/r06_lsq_rotation.txt).  Each wave still sums its own tiles in sweep order:
  // deterministic, the same in every variant of a shape.
  int64_t org = 0;
  int rot = blk;
  const int grid1 = a.grid;
  if constexpr (MODE & M_BLOCKED) {
    const int64_t tile = int64_t(kWaves) * RB;
    const int64_t per = ((rows + a.grid - 1) / a.grid + tile - 1) / tile * tile;
    const int64_t lo = int64_t(blk) * per;
    hi = lo + per < rows ? lo + per : rows;
    step = tile;
    base = lo + int64_t(wave) * RB;
  } else {
    step = int64_t(a.grid) * kWaves * RB;
    base = (int64_t(blk) * kWaves + wave) * RB;
    hi = rows;
  }
  // the wave's next tile (bases strictly increase, so the first one past hi ends the loop)
  auto nxt = [&]() -> int64_t {
    if constexpr ((MODE & M_BLOCKED) || !(MODE & M_ROTATE)) {
      base += step;
    } else {
      org += step;
      rot = rot + 1 == grid1 ? 0 : rot + 1;
      base = org + (int64_t(rot) * kWaves + wave) * RB;
    }
    return base;
  };

  // Fused head: workgroup 0 runs this epoch's coordinator step; its dispatch copies (the
  // messages the tasks read) are stored write-through, the others' first tile of A is in
  // flight while they wait for its token, and they read their message write-through too (the
  // tree's hand-off: no L2 writeback / invalidate).
  [[maybe_unused]] bool pre = false;
  Tile<T, VPL, RB, MODE> t0;
  if constexpr ((MODE & M_HEAD) != 0) {
    if (blockIdx.x == 0) {
      // (the step reads its arguments from the kernel arguments or from LDS in two separate
      // calls: one pointer that may point at either made the compiler copy the 976-B kernarg
      // EpochArgs to scratch, 3.5 KiB of it per workgroup and 50 us per launch)
      if (batch.head & kHeadPrearmed) {
        // pre-armed: the host decides this epoch while the launch waits here; the step's
        // arguments then come from the pinned mailbox (one pass of 16-B reads into LDS)
        __shared__ EpochArgs s_ep;
        __shared__ int s_go;
        // the launch's own arguments into LDS while the host decides: when its prediction holds
        // (kPreSame, most epochs) the step starts the moment the go word lands
        constexpr int kEpVecs = int(sizeof(EpochArgs) / 16);
        static_assert(sizeof(EpochArgs) % 16 == 0, "EpochArgs copies in 16-B vectors");
        for (int k = tid; k < kEpVecs; k += kThreads)
          reinterpret_cast<uint4*>(&s_ep)[k] = reinterpret_cast<const uint4*>(&batch.ep)[k];
        if (tid == 0) {
          const unsigned long long t0s = rt_now();
          int go = 1;
          unsigned long long v;
          for (unsigned k = 0; ((v = __hip_atomic_load(batch.pre_go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) &
                                ~(kPreCancel | kPreSame)) != batch.pre_token;
               ++k) {
            if ((k & 255) == 255 && rt_now() - t0s > batch.spin_ticks) {
              __hip_atomic_fetch_or(batch.err, 128u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              v = kPreCancel;
              break;
            }
          }
          if (v & kPreCancel) go = 0;
          else if (v & kPreSame) go = 2;
          MPA_HEAD_STAMP(batch.head_token, 0, false);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the mailbox the host wrote
          s_go = go;
        }
        __syncthreads();
        if (!s_go) {
          if (tid == 0)
            __hip_atomic_store(batch.head_word, batch.head_token | kHeadCancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return;
        }
        // a changed decision: the arguments from the mailbox over the bus
        if (s_go == 1) {
          const uint4* src = reinterpret_cast<const uint4*>(batch.pre_ep);
          for (int k = tid; k < kEpVecs; k += kThreads) reinterpret_cast<uint4*>(&s_ep)[k] = src[k];
          __syncthreads();
        }
        if (tid == 0) MPA_HEAD_STAMP(batch.head_token, 5, false);
        if ((batch.head & 3) == 2) epoch_elems<T, E, true, false>(s_ep, tid, kThreads);
        else epoch_elems<T, 1, true, false>(s_ep, tid, kThreads);
        if (tid == 0) MPA_HEAD_STAMP(batch.head_token, 6, false);
      } else if ((batch.head & 3) == 2) {
        epoch_elems<T, E, true, false>(batch.ep, tid, kThreads);
      } else {
        epoch_elems<T, 1, true, false>(batch.ep, tid, kThreads);
      }
      drain_vm();
      __syncthreads();
      if (tid == 0) {
        __hip_atomic_store(batch.head_word, batch.head_token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        MPA_HEAD_STAMP(batch.head_token, 1, false);
      }
    } else {
      if (base < hi) {
        t0.load(A, base, rows, a.lda, lane, vok);
        t0.load_b(bv, base, rows);
        pre = true;
      }
      if (tid == 0) {
        const unsigned long long t0s = rt_now();
        s_ticket = 1;
        // a pre-armed launch waits for the host's decision first: no time bound of its own
        // here beyond workgroup 0's (which publishes the cancel token on its timeout)
        for (unsigned k = 0;; ++k) {
          const uint32_t hw = __hip_atomic_load(batch.head_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (hw == batch.head_token) {
            MPA_HEAD_STAMP(batch.head_token, 2, true);
            break;
          }
          if (hw == (batch.head_token | kHeadCancel)) {
            s_ticket = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if ((k & 255) == 255 && rt_now() - t0s > 2 * batch.spin_ticks) {
            __hip_atomic_fetch_or(batch.err, 128u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            s_ticket = 0;  // no work: the host watchdog reports the error word
            break;
          }
        }
      }
      __syncthreads();
      if (!s_ticket) return;
    }
  }
  if constexpr ((MODE & M_HEAD) != 0) {
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int c0 = (v * 64 + lane) * E;
#pragma unroll
      for (int e = 0; e < E; ++e) xr[v].v[e] = (c0 + e < a.cols) ? ld_agent(xv + c0 + e) : T(0);
    }
  }

  if constexpr (MODE & M_PREFETCH) {
    Tile<T, VPL, RB, MODE> t1;
    if (base < hi && !pre) {
      t0.load(A, base, rows, a.lda, lane, vok);
      t0.load_b(bv, base, rows);
    }
    for (;;) {
      const int64_t b0 = base;
      if (b0 >= hi) break;
      const int64_t b1 = nxt();
      if (b1 < hi) {
        t1.load(A, b1, rows, a.lda, lane, vok);
        t1.load_b(bv, b1, rows);
      }
      t0.compute(bv, b0, rows, xr, g);
      if (b1 >= hi) break;
      const int64_t b2 = nxt();
      if (b2 < hi) {
        t0.load(A, b2, rows, a.lda, lane, vok);
        t0.load_b(bv, b2, rows);
      }
      t1.compute(bv, b1, rows, xr, g);
    }
  } else if constexpr ((MODE & M_HEAD) != 0) {
    for (; base < hi; nxt()) {
      if (!pre) {
        t0.load(A, base, rows, a.lda, lane, vok);
        t0.load_b(bv, base, rows);
      }
      pre = false;
      t0.compute(bv, base, rows, xr, g);
    }
  } else {
    for (; base < hi; nxt()) {
      Tile<T, VPL, RB, MODE> t;
      t.load(A, base, rows, a.lda, lane, vok);
      t.compute(bv, base, rows, xr, g);
    }
  }

  MPA_LSQ_WG_STAMP(1);
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
  // Cross-workgroup reduction: a fan-in-8 tree over the workgroup partials, with no
  // waiting.  Level l groups 8 consecutive level-l partials; the member that arrives LAST
  // at its group's counter sums the group in member order and carries the result to level
  // l+1; the others return.  Partials are stored and loaded write-through (st_sc1 /
  // ld_sc1), so the hand-offs need no fences.  A workgroup
  // only ever reads partials whose writers have already arrived, so the tree completes
  // whatever the residency (concurrent launches of delayed workers filled the chip with
  // spinning reducers under the earlier wait-for-all scheme: fp64, 2048 columns, 8
  // concurrent single-task launches ran 1000x slow).  Partials stay in place: the level-l
  // partial of element e sits in slab row e * 8^l; each counter is reset by its group's
  // last arriver, and the next launch of the worker is stream-ordered after this one.
  constexpr int S = VPL * 64;  // 16-B vectors per partial
  constexpr unsigned F = kLsqFanIn;
  P* __restrict__ slab = static_cast<P*>(a.slab);
  T* __restrict__ out = static_cast<T*>(a.out);
  const unsigned G = unsigned(a.grid);
  // a reply that stays on this GPU is stored write-through (publish_done_wt needs no release)
  auto store_out = [&](int j, const P& s) {
    const int c0 = j * E;
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (c0 + e < a.cols) {
        if (a.pub_local) st_agent(out + c0 + e, s.v[e]);
        else out[c0 + e] = s.v[e];
      }
  };
  bool cx = false;  // cancelled (read by the reply's writer only)
  // One-level tree for small partials (one 16-B vector per lane, <= 64 workgroups: c1's tasks):
  // every workgroup stores its partial and counts in; the last one sums all G of them, four
  // threads per vector each over every fourth partial in order, then the four sums in order
  // in LDS -- one counter round trip and one load round instead of two of each.
  constexpr bool kOneLevel = (S == 64) && (MODE & M_PREFETCH) == 0 && (MODE & M_TREE_FENCE) == 0;
  if (kOneLevel && G > 1 && G <= 64) {
    for (int j = tid; j < S; j += kThreads) st_sc1(&slab[size_t(blk) * S + j], red[j]);
    drain_vm();
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(&a.ctr[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_ticket = old + 1 == G;
      if (s_ticket) __hip_atomic_store(&a.ctr[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_ticket) return;
    if constexpr ((MODE & M_HEAD) != 0)
      if (tid == 0) MPA_HEAD_STAMP(batch.head_token, 3, true);
    const int j = tid & (S - 1), q = tid / S;  // kThreads = 4 * S: four partial sums per vector
    P acc;
#pragma unroll
    for (int e = 0; e < E; ++e) acc.v[e] = T(0);
    // clamped, every load issues at once (each one under its own branch was waited for there:
    // up to 16 round trips in a row for the last reducer of a 64-workgroup task)
    P t[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int p = q + 4 * m < int(G) ? q + 4 * m : int(G) - 1;
      t[m] = ld_sc1(&slab[size_t(p) * S + j]);
    }
    // the cancel word (pinned host memory: a PCIe round trip) read while the partials' loads are
    // in flight, not before they issue
    cx = cancelled();
#pragma unroll
    for (int m = 0; m < 16; ++m)
      if (q + 4 * m < int(G))
#pragma unroll
        for (int e = 0; e < E; ++e) acc.v[e] = m == 0 ? t[m].v[e] : acc.v[e] + t[m].v[e];
    __syncthreads();  // red[] is free again: the four sums of every vector
    if (q > 0) red2[(q - 1) * S + j] = acc;
    __syncthreads();
    if (q == 0 && !cx) {
#pragma unroll
      for (int r = 0; r < 3; ++r)
        if (r + 1 < int(G))
#pragma unroll
          for (int e = 0; e < E; ++e) acc.v[e] += red2[r * S + j].v[e];
      store_out(j, acc);
    }
  } else if (G == 1) {
    cx = cancelled();
    if (!cx)
      for (int j = tid; j < S; j += kThreads) store_out(j, red[j]);
  } else {
    constexpr bool FENCE = (MODE & M_TREE_FENCE) != 0;
    auto put = [&](P* d, const P& v) {
      if constexpr (FENCE) *d = v;
      else st_sc1(d, v);
    };
    auto get = [&](const P* q) -> P {
      if constexpr (FENCE) return *q;
      else return ld_sc1(q);
    };
    for (int j = tid; j < S; j += kThreads) put(&slab[size_t(blk) * S + j], red[j]);
    unsigned idx = unsigned(blk), count = G, stride = 1;
    int lvl_off = 0, lvl_cap = kLsqMaxGrid / int(F);
    for (;;) {
      drain_vm();
      __syncthreads();
      const unsigned first = (idx / F) * F;
      const unsigned gsize = count - first < F ? count - first : F;
      if (tid == 0) {
        unsigned* c = &a.ctr[lvl_off + int(idx / F)];
        if constexpr (FENCE) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          drain_vm();
        }
        const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_ticket = old + 1 == gsize;
        if (s_ticket) {
          __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if constexpr (FENCE) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            drain_vm();
          }
        }
      }
      __syncthreads();
      if (!s_ticket) return;  // an earlier arriver of the group: the last one carries it
      const unsigned next = (count + F - 1) / F;
      if (next == 1) cx = cancelled();
      if (next == 1 && tid == 0) MPA_LSQ_MAX_STAMP(g_lsq_root);
      const P* src = slab + size_t(first) * stride * S;
      for (int j = tid; j < S; j += kThreads) {
        P t[F];
#pragma unroll
        for (unsigned m = 0; m < F; ++m)
          if (m < gsize) t[m] = get(&src[size_t(m) * stride * S + j]);
        P s = t[0];
#pragma unroll
        for (unsigned m = 1; m < F; ++m)
          if (m < gsize)
#pragma unroll
            for (int e = 0; e < E; ++e) s.v[e] += t[m].v[e];
        if (next == 1) {
          if (!cx) store_out(j, s);
        } else {
          put(&slab[size_t(first) * stride * S + j], s);
        }
      }
      if (next == 1) break;
      idx /= F;
      count = next;
      stride *= F;
      lvl_off += lvl_cap;
      lvl_cap = (lvl_cap + int(F) - 1) / int(F);
    }
  }
  drain_vm();
  __syncthreads();
  if (cx) return;
  if (tid == 0) {
    if constexpr ((MODE & M_HEAD) != 0) MPA_HEAD_STAMP(batch.head_token, 4, false);
    if (a.pub_local) publish_done_wt(a.flag, a.seq);
    else publish_done(a.flag, a.seq);
    publish_peer(a.flag2, a.seq);
    MPA_LSQ_MAX_STAMP(g_lsq_pub);
  }
  if (!batch.tail) return;
  // Fused tail: this workgroup finished its task (and published it); the last task of the
  // launch to finish runs the next epoch's coordinator step.  publish_done released the
  // reply chunk before the count; the last counter acquires the others' chunks.
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(batch.tail_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_ticket = old + 1 == unsigned(batch.ntasks);
    if (s_ticket) {
      __hip_atomic_store(batch.tail_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
  }
  __syncthreads();
  if (!s_ticket) return;
  if (batch.tail_nwait > 0) {
    // the workers served by other processes: wave 0 polls their completion words (lane k:
    // word k, relaxed system-scope loads of the shared mailbox), as wait_words_kernel does
    if (tid < 64) {
      const int k = tid;
      bool ok = k >= batch.tail_nwait;
      const unsigned long long t0 = rt_now();
      for (unsigned it = 0;; ++it) {
        if (!ok) ok = __hip_atomic_load(batch.tail_word[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= batch.tail_target[k];
        if (__builtin_amdgcn_ballot_w64(!ok) == 0ull) break;
        __builtin_amdgcn_s_sleep(2);
        if ((it & 63) == 63 && rt_now() - t0 > batch.spin_ticks) {
          if (k == 0) __hip_atomic_fetch_or(batch.err, 32u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          s_ticket = 0;  // no step: the host watchdog reports the error word
          break;
        }
      }
    }
    __syncthreads();
    if (!s_ticket) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the replies the remote tasks released
  } else {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  if (batch.tail == 2) epoch_elems<T, E, false, false>(batch.ep, tid, kThreads);
  else epoch_elems<T, 1, false, false>(batch.ep, tid, kThreads);
  if (batch.ep.ndoor == 0) return;
  // the next messages of remote workers are in their slots (written through at system scope,
  // EpochArgs::dst_sys; or plain and released here, sys_fence): ring the doorbells (as
  // epoch_kernel's last block)
  drain_vm();
  __syncthreads();
  if (tid == 0) {
    if (batch.ep.sys_fence) {
      __threadfence_system();
      drain_vm();
      for (int d = 0; d < batch.ep.ndoor; ++d)
        __hip_atomic_store(batch.ep.door[d], batch.ep.doorval[d], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      for (int d = 0; d < batch.ep.ndoor; ++d)
        __hip_atomic_store(batch.ep.door[d], batch.ep.doorval[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <typename T, int VPL, int RB, int MODE>
hipError_t go(const LsqBatch& a, hipStream_t s) {
  const int grid = a.block0[a.ntasks];
  if (grid <= 0) return hipSuccess;
  if (batch_armed(a)) hipLaunchKernelGGL((lsq_grad_kernel<T, VPL, RB, MODE | M_ARMED>), dim3(grid), dim3(kThreads), 0, s, a);
  else if (a.head) hipLaunchKernelGGL((lsq_grad_kernel<T, VPL, RB, MODE | M_HEAD>), dim3(grid), dim3(kThreads), 0, s, a);
  else hipLaunchKernelGGL((lsq_grad_kernel<T, VPL, RB, MODE>), dim3(grid), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

template <typename T>
constexpr int vpl_for(int cols) {
  constexpr int per = 64 * Pack<T>::E;
  return (cols + per - 1) / per;
}

// tuning variants of the BASELINE c2 shape (fp32, 1024 columns), selectable with
// MPA_LSQ_VARIANT=<index> for measurement; kDefaultC2 is the one shipped
using Launch = hipError_t (*)(const LsqBatch&, hipStream_t);
struct Variant {
  Launch fn;
  int rb;
  const char* name;
};
constexpr Variant kC2Variants[] = {
    // shipped: 6.5 TB/s on c2 in the round-1 sweep (profiles/r01_tune_sweep*.jsonl)
    {go<float, 4, 4, M_CLAMP | M_DPP | M_NT | M_ROTATE>, 4, "rb4+clamp+dpp+nt+rotate"},
#if MPA_MEASURE
    {go<float, 4, 4, M_CLAMP | M_DPP | M_NT>, 4, "rb4+clamp+dpp+nt (round 5's, no rotation)"},
    // the tuning space of that sweep (measurement build only: make MEASURE=1)
    {go<float, 4, 4, 0>, 4, "rb4"},
    {go<float, 4, 4, M_CLAMP>, 4, "rb4+clamp"},
    {go<float, 4, 4, M_CLAMP | M_DPP>, 4, "rb4+clamp+dpp"},
    {go<float, 4, 2, M_CLAMP | M_DPP | M_PREFETCH>, 2, "rb2+clamp+dpp+prefetch"},
    {go<float, 4, 4, M_CLAMP | M_DPP | M_PREFETCH>, 4, "rb4+clamp+dpp+prefetch"},
    {go<float, 4, 2, M_CLAMP | M_DPP | M_PREFETCH | M_NT>, 2, "rb2+clamp+dpp+prefetch+nt"},
    {go<float, 4, 8, M_CLAMP | M_DPP>, 8, "rb8+clamp+dpp"},
    {go<float, 4, 2, M_CLAMP | M_DPP>, 2, "rb2+clamp+dpp"},
    {go<float, 4, 4, M_CLAMP | M_DPP | M_NT | M_TREE_FENCE>, 4, "rb4+clamp+dpp+nt+fenced-tree"},
    {go<float, 4, 4, M_CLAMP | M_DPP | M_NT | M_BLOCKED>, 4, "rb4+clamp+dpp+nt+blocked"},
    {go<float, 4, 2, M_CLAMP | M_DPP | M_PREFETCH | M_NT | M_BLOCKED>, 2, "rb2+clamp+dpp+prefetch+nt+blocked"},
    {go<float, 4, 4, M_CLAMP | M_DPP | M_PREFETCH | M_NT | M_BLOCKED>, 4, "rb4+clamp+dpp+prefetch+nt+blocked"},
    {go<float, 4, 8, M_CLAMP | M_DPP | M_NT | M_BLOCKED>, 8, "rb8+clamp+dpp+nt+blocked"},
    // round 5: 32 KiB per wave and tile, as the batched 2048-column launch (profiles/r05_lsq2048.txt)
    {go<float, 4, 8, M_CLAMP | M_DPP | M_NT>, 8, "rb8+clamp+dpp+nt"},
    {go<float, 4, 6, M_CLAMP | M_DPP | M_NT>, 6, "rb6+clamp+dpp+nt"},
#endif
};
constexpr int kNumC2Variants = int(sizeof(kC2Variants) / sizeof(kC2Variants[0]));
constexpr int kDefaultC2 = 0;

int g_variant = -1;  // set by MPA_LSQ_VARIANT or mpa_tune("lsq_variant", i)

int c2_variant() {
  if (g_variant < 0) {
    const char* e = std::getenv("MPA_LSQ_VARIANT");
    const int i = e ? std::atoi(e) : kDefaultC2;
    g_variant = (i >= 0 && i < kNumC2Variants) ? i : kDefaultC2;
  }
  return g_variant;
}

constexpr int kMode = M_CLAMP | M_DPP | M_NT;  // shipped mode of the other shapes

// rows per wave iteration of the fp64 <= 128-column shape (c1: 4096 x 64 per worker): 16, so
// a wave's whole share of a c1 task is in flight at once (c1 56-57k against 53-54k it/s with 4,
// profiles/r03_c1_rb_ab.txt; 4 and 8 stay selectable in the measurement build)
int small_f64_rb() {
#if MPA_MEASURE
  static const int rb = [] {
    const char* e = std::getenv("MPA_LSQ_SMALL_RB");
    const int v = e ? std::atoi(e) : 16;
    return v == 4 || v == 8 ? v : 16;
  }();
  return rb;
#else
  return 16;
#endif
}

}  // namespace

int lsq_cols_pad(int dtype, int cols) {
  if (cols <= 0) return 0;
  if ((dtype == MPA_F32 || dtype == MPA_F64) && cols > kLsqWideSlice)  // wide: whole slices
    return cols <= kLsqWideMaxCols ? (cols + kLsqWideSlice - 1) / kLsqWideSlice * kLsqWideSlice : 0;
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

int lsq_rows_per_wave_iter(int dtype, int cols) {
  const int cp = lsq_cols_pad(dtype, cols);
  if (cp > kLsqWideSlice) return 1;
  if (dtype == MPA_F32) {
    if (cp == 1024) return kC2Variants[c2_variant()].rb;
    return cp < 1024 ? 4 : 2;
  }
  if (cp == 128) return small_f64_rb();
  return cp <= 256 ? 4 : cp <= 1024 ? 2 : 1;
}

#if MPA_MEASURE
// the 2048-column shapes of c3 / c4 (measurement build, MPA_LSQ_V2048=<index>; 0 = shipped)
static int v2048() {
  static const int v = [] {
    const char* e = std::getenv("MPA_LSQ_V2048");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}
#endif

const char* lsq_variant_name() { return kC2Variants[c2_variant()].name; }

#if MPA_MEASURE
// MPA_LSQ_STAMP=1 (measurement build): the last lsq_grad_kernel launch's timeline, from its first
// workgroup's entry (us): the last entry, the block loops' ends (median, last), the last tree
// root's start and the last publish
void lsq_stamp_dump() {
  static unsigned long long wg[kLsqStampWgs][4];
  static unsigned xcc[kLsqStampWgs];
  unsigned long long root = 0, pub = 0;
  unsigned grid = 0;
  if (hipMemcpyFromSymbol(wg, HIP_SYMBOL(g_lsq_wg), sizeof(wg)) != hipSuccess ||
      hipMemcpyFromSymbol(&root, HIP_SYMBOL(g_lsq_root), sizeof(root)) != hipSuccess ||
      hipMemcpyFromSymbol(&pub, HIP_SYMBOL(g_lsq_pub), sizeof(pub)) != hipSuccess ||
      hipMemcpyFromSymbol(&grid, HIP_SYMBOL(g_lsq_grid), sizeof(grid)) != hipSuccess ||
      hipMemcpyFromSymbol(xcc, HIP_SYMBOL(g_lsq_xcc), sizeof(xcc)) != hipSuccess)
    return;
  const unsigned n = grid < unsigned(kLsqStampWgs) ? grid : unsigned(kLsqStampWgs);
  if (!n) return;
  unsigned long long t0 = ~0ull, s1 = 0;
  std::vector<double> ends;
  for (unsigned b = 0; b < n; ++b) {
    t0 = std::min(t0, wg[b][0]);
    s1 = std::max(s1, wg[b][0]);
  }
  for (unsigned b = 0; b < n; ++b) ends.push_back(double(wg[b][1] - t0) / 100.0);
  std::sort(ends.begin(), ends.end());
  std::fprintf(stderr, "[mpa lsq stamps] last launch, %u workgroups (us from the first entry): last entry %.2f, "
               "loop ends p10 %.2f median %.2f last %.2f, last tree root %.2f, last publish %.2f\n", n,
               double(s1 - t0) / 100.0, ends[n / 10], ends[n / 2], ends.back(), double(root - t0) / 100.0,
               double(pub - t0) / 100.0);
  // by blockIdx % 8 (the XCD under round-robin placement): median and last loop end
  std::fprintf(stderr, "[mpa lsq stamps] loop ends by workgroup %% 8 (median / last):");
  for (unsigned x = 0; x < 8; ++x) {
    std::vector<double> e;
    for (unsigned b = x; b < n; b += 8) e.push_back(double(wg[b][1] - t0) / 100.0);
    if (e.empty()) continue;
    std::sort(e.begin(), e.end());
    std::fprintf(stderr, " %u: %.1f / %.1f", x, e[e.size() / 2], e.back());
  }
  std::fprintf(stderr, "\n");
  // the shader clock over each workgroup's block loop (s_memtime cycles / s_memrealtime at 100 MHz)
  std::fprintf(stderr, "[mpa lsq stamps] loop clock GHz by workgroup %% 8 (median):");
  for (unsigned x = 0; x < 8; ++x) {
    std::vector<double> c;
    for (unsigned b = x; b < n; b += 8)
      if (wg[b][1] > wg[b][0]) c.push_back(double(wg[b][3] - wg[b][2]) / double(wg[b][1] - wg[b][0]) * 0.1);
    if (c.empty()) continue;
    std::sort(c.begin(), c.end());
    std::fprintf(stderr, " %u: %.3f", x, c[c.size() / 2]);
  }
  std::fprintf(stderr, "\n");
  // by the XCC the workgroup actually ran on: how many, loop end median, clock median; and how
  // many workgroups ran on XCC (blockIdx % 8)
  unsigned match = 0;
  for (unsigned b = 0; b < n; ++b) match += xcc[b] == b % 8;
  std::fprintf(stderr, "[mpa lsq stamps] by XCC (workgroups, loop end median, clock GHz median); %u of %u on XCC blockIdx %% 8:",
               match, n);
  for (unsigned x = 0; x < 8; ++x) {
    std::vector<double> e, c;
    for (unsigned b = 0; b < n; ++b)
      if (xcc[b] == x) {
        e.push_back(double(wg[b][1] - t0) / 100.0);
        if (wg[b][1] > wg[b][0]) c.push_back(double(wg[b][3] - wg[b][2]) / double(wg[b][1] - wg[b][0]) * 0.1);
      }
    if (e.empty()) continue;
    std::sort(e.begin(), e.end());
    std::sort(c.begin(), c.end());
    std::fprintf(stderr, " %u: %zu %.1f %.3f", x, e.size(), e[e.size() / 2], c.empty() ? 0.0 : c[c.size() / 2]);
  }
  std::fprintf(stderr, "\n");
}
#endif

#if MPA_MEASURE
void head_stamp_reset() {
  static unsigned long long h[kHeadSlots][7];
  for (int i = 0; i < kHeadSlots; ++i) {
    h[i][0] = h[i][1] = h[i][3] = h[i][4] = h[i][5] = h[i][6] = 0;
    h[i][2] = ~0ull;
  }
  h[0][3] = ~0ull;
  for (int i = 0; i < kHeadSlots; ++i) h[i][3] = ~0ull;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_head_stamp), h, sizeof(h));
}
void head_stamp_dump() {
  static unsigned long long h[kHeadSlots][7];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_head_stamp), sizeof(h)) != hipSuccess) return;
  std::vector<double> d[9];
  for (int i = 1; i < kHeadSlots; ++i) {
    const auto* a = h[i];
    const auto* p = h[i - 1];
    if (!a[0] || !a[1] || a[2] == ~0ull || a[3] == ~0ull || !a[4]) continue;
    d[0].push_back(double(a[1] - a[0]) / 100.0);  // 100 MHz realtime -> us
    d[1].push_back(double(a[2] - a[1]) / 100.0);
    d[2].push_back(double(a[3]) / 100.0 - double(a[2]) / 100.0);
    d[3].push_back(double(a[4]) / 100.0 - double(a[3]) / 100.0);
    d[4].push_back(double(a[4] - a[0]) / 100.0);
    if (p[4] && p[4] < a[0]) d[5].push_back(double(a[0] - p[4]) / 100.0);  // previous publish -> this go
    if (a[5] && a[6]) {  // the pre-armed head's step, split
      d[6].push_back(double(a[5]) / 100.0 - double(a[0]) / 100.0);
      d[7].push_back(double(a[6]) / 100.0 - double(a[5]) / 100.0);
      d[8].push_back(double(a[1]) / 100.0 - double(a[6]) / 100.0);
    }
  }
  static const char* names[9] = {"go seen -> head token", "head token -> seen by another WG", "token seen -> first task's last reducer",
                                 "last reducer -> last publish", "go seen -> last publish (device part)", "previous epoch's last publish -> go seen",
                                 "  go seen -> step start (acquire, arguments)", "  step start -> step's stores issued", "  stores issued -> head token (drain)"};
  std::fprintf(stderr, "[mpa head stamps] %zu launches, %zu with the step split (us, p10 / p50 / p90):\n", d[4].size(), d[6].size());
  for (int k = 0; k < 9; ++k) {
    if (d[k].empty()) continue;
    std::sort(d[k].begin(), d[k].end());
    const size_t n = d[k].size();
    std::fprintf(stderr, "  %-44s %6.2f %6.2f %6.2f\n", names[k], d[k][n / 10], d[k][n / 2], d[k][n * 9 / 10]);
  }
}
#endif

int lsq_set_variant(int i) {
  if (i < 0 || i >= kNumC2Variants) return -1;
  g_variant = i;
  return kNumC2Variants;
}

hipError_t launch_lsq(int dtype, int cols, const LsqBatch& a, hipStream_t s) {
  const int cp = lsq_cols_pad(dtype, cols);
  if (cp > kLsqWideSlice) return launch_lsqw(dtype, a, s);
  if (dtype == MPA_F32) {
    switch (cp) {
      case 256: return go<float, 1, 4, kMode>(a, s);
      case 512: return go<float, 2, 4, kMode>(a, s);
      case 1024: return kC2Variants[c2_variant()].fn(a, s);
      case 2048:
#if MPA_MEASURE
        switch (v2048()) {
          case 1: return go<float, 8, 1, kMode>(a, s);
          case 2: return go<float, 8, 4, kMode>(a, s);
          case 3: return go<float, 8, 2, kMode | M_PREFETCH>(a, s);
          case 4: return go<float, 8, 1, kMode | M_PREFETCH>(a, s);
          case 5: return go<float, 8, 2, kMode | M_BLOCKED>(a, s);
          case 6: return go<float, 8, 4, kMode | M_BLOCKED>(a, s);
          default: break;
        }
#endif
        // a batched launch of several tasks (one grid for all of them: nwait = n, no delays)
        // streams 32 KiB per wave and tile: the c3 tasks batched (measurement config c3k) 0.76
        // -> 0.83-0.90 of HBM, and so does a lone task of a process that serves one worker (the
        // node's N = 8 placement, measurement config c3n8: 0.76 -> 0.88, profiles/r06_pergpu.txt);
        // one task per launch beside others (c3's delayed tasks at N = 1, two to four launches
        // overlapping) keeps 16 KiB and three waves per SIMD: -4 % with four rows
        // (profiles/r05_lsq2048.txt)
        if (a.ntasks >= 2 || a.alone) return go<float, 8, 4, kMode>(a, s);
        return go<float, 8, 2, kMode>(a, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (dtype == MPA_F64) {
    switch (cp) {
      case 128:
#if MPA_MEASURE
        if (small_f64_rb() == 4) return go<double, 1, 4, kMode>(a, s);
        if (small_f64_rb() == 8) return go<double, 1, 8, kMode>(a, s);
#endif
        return go<double, 1, 16, kMode>(a, s);
      case 256: return go<double, 2, 4, kMode>(a, s);
      case 512: return go<double, 4, 2, kMode>(a, s);
      case 1024: return go<double, 8, 2, kMode>(a, s);
      case 2048:
#if MPA_MEASURE
        switch (v2048()) {
          case 1: return go<double, 16, 1, kMode | M_PREFETCH>(a, s);
          case 2: return go<double, 16, 2, kMode>(a, s);
          case 3: return go<double, 16, 1, kMode | M_BLOCKED>(a, s);
          case 4: return go<double, 16, 1, M_CLAMP | M_DPP>(a, s);
          default: break;
        }
#endif
        return go<double, 16, 1, kMode>(a, s);
      default: return hipErrorInvalidValue;
    }
  }
  return hipErrorInvalidValue;
}

}  // namespace mpa
