// Host-callable launchers of the gfx950 kernels (kernels.hip).  All launches are
// asynchronous on the given stream; shapes are validated by the caller (transport_hip.cpp)
// before a launch, so a kernel never indexes outside the buffers it is given.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mpa {

// One flush of the pool = ONE exchange launch: a list of byte copies (sendbuf -> isendbuf
// slots, sendbuf -> remote workers' mailboxes, irecvbuf/mailbox replies -> recvbuf
// chunks) and, once every copy of the launch is complete and released at system scope,
// the doorbells of the remote workers it posted to (rung by the last block to finish).
constexpr int kMaxCopies = 48;
constexpr int kMaxDoorbells = 16;
struct CopyItem {
  const uint8_t* src;
  uint8_t* dst;
  uint64_t bytes;
};
struct ExchangeArgs {
  int ncopy, ndoor;
  uint64_t part;  // bytes per block (multiple of 16)
  int block0[kMaxCopies + 1];
  CopyItem c[kMaxCopies];
  unsigned long long* door[kMaxDoorbells];
  unsigned long long doorval[kMaxDoorbells];
  uint32_t* ticket;      // monotonic block counter in device memory (doorbell launches only)
  uint32_t ticket_base;  // its value before this launch
};
hipError_t launch_exchange(const ExchangeArgs& a, hipStream_t s);

// rank 0's wait for the completion words of the remote workers of a launched-ahead epoch:
// ONE single-wave launch that polls every word (lane j: word j, system-scope loads of the
// shared-memory mailbox) until each reaches its target, then acquires at system scope.  It
// replaces one hipStreamWaitValue64 per remote worker (each a blit kernel of its own, ~4-5 us
// apiece in series on the coordinator stream: 7 of them per epoch at N = 8).  Bounded:
// past spin_ticks it sets err bit 32 and returns.
constexpr int kMaxWaitWords = 64;
struct WaitWordsArgs {
  int n;
  const unsigned long long* word[kMaxWaitWords];
  unsigned long long target[kMaxWaitWords];
  unsigned int* err;
  unsigned long long spin_ticks;
};
hipError_t launch_wait_words(const WaitWordsArgs& a, hipStream_t s);

// completion protocol shared by every worker task kernel
struct Publish {
  unsigned long long* flag;  // host-pinned: seq of the last completed task of the worker
  unsigned int* err;         // host-pinned: first device-side error code (0 = none)
  unsigned long long seq;
  unsigned long long spin_ticks;  // bound on any in-kernel wait (s_memrealtime ticks)
};

// One coordinator epoch step as ONE launch (the native descent loop): the
// pending harvest copies `recvbufs[i] .= irecvbufs[i]` of the previous call, the iterate
// update x -= eta * sum_i w_i chunk_i (the user code between two asyncmap! calls,
// examples/iterative_example.jl:41-46), the harvests of this call's phase 1, and the
// dispatch copies `isendbufs[i] .= sendbuf` (:130) of the updated iterate, then the
// doorbells of remote workers.  Element-parallel: element j of every chunk, of x and of
// every message is handled by one thread, so the stages need no grid-wide ordering.
constexpr int kMaxEpochChunks = 16;
constexpr int kMaxEpochDst = 32;
constexpr int kMaxEpochDst0 = 8;
struct EpochArgs {
  int64_t elems;  // elements per chunk (T) = per message
  int n;          // chunks of recvbuf
  int update;     // 0: no update stage (the message is x as it stands)
  uint8_t* recv;  // recvbuf, chunk i at i * elems
  const uint8_t* hsrc[kMaxEpochChunks];   // harvest source of chunk i before the update (NULL: none)
  const uint8_t* hsrc2[kMaxEpochChunks];  // harvest source of chunk i after it
  double w[kMaxEpochChunks];
  double eta;
  void* x;           // T[elems], updated in place
  uint16_t* mirror;  // bf16 copy of the updated x (batched variant) or NULL
  int msg_bf16;      // the message is the bf16 mirror (else x)
  int ndst;
  uint8_t* dst[kMaxEpochDst];
  int ndoor;
  // dispatch copies of the iterate as it stands BEFORE the update: the stale re-dispatches
  // held by the previous call's wait (flush_stale deferred their messages into this step)
  int ndst0;
  uint8_t* dst0[kMaxEpochDst0];
  unsigned long long* door[kMaxDoorbells];
  unsigned long long doorval[kMaxDoorbells];
  uint32_t* ticket;
  uint32_t ticket_base;
  // messages other processes read (remote workers' slots): bit k set = dst[k] is stored
  // write-through at system scope (sc0 sc1), so the doorbells need no L2 writeback; sys_fence
  // = 1 (MPA_MSG_WT=0): plain stores and a system-scope release in every workgroup instead
  uint32_t dst_sys;
  uint32_t sys_fence;
  uint32_t reserved_[3];
};
// One worker task of a least-squares launch.
struct LsqTask {
  const void* A;
  const void* b;
  const void* x;
  void* out;
  void* slab;       // [grid][cols_pad] partial sums (T), reduced in place
  uint32_t* ctr;    // [kLsqCtrPerTask] reduction-tree arrival counters, zero between launches
  unsigned long long* flag;  // host-pinned completion word of the worker
  unsigned long long* flag2;  // N > 1, a worker process's task: rank 0's device copy of the done word, or null
  unsigned long long seq;
  int64_t rows, lda;
  int cols, grid;
  // pre-armed launch of a worker process: the server's cancel word; equal
  // to seq means "disarmed", and the task returns without computing or publishing (NULL:
  // not armed)
  const unsigned long long* go;
  // device-armed launch of a worker process: the worker's doorbell word in this GPU's
  // message slot, which rank 0 rings over xGMI; every workgroup waits for it to reach seq
  // before any work (wait_door, device_common.hpp).  NULL: launched when rung
  const unsigned long long* door;
  // wide rows (cols > 2048, lsqw_kernel.hip): the residual r = A x - b (rows T), the
  // per-slice tree and slice-completion counters, and the row groups of the second pass
  void* r;
  uint32_t* wctr;
  int grid2;
  int pub_local;  // the reply stays on this GPU: publish_done_local (device_common.hpp)
};
// Wide rows: two passes (r = A x - b, then g = A^T r over 2048-column slices), A read twice.
constexpr int kLsqWideSlice = 2048;   // columns per slice (fp32: 8 x 16 B per lane, fp64: 16)
constexpr int kLsqWideMaxCols = 65536;
constexpr int kLsqWideMaxGroups = 64;  // row groups per slice in the second pass (fan-in-8 tree)
constexpr int kLsqWideCtrPerSlice = 16;
constexpr unsigned long long kCancelBit = 1ull << 62;

// Reduction tree of a least-squares task (lsq_kernel.hip): fan-in, most workgroups per
// task, and the counters it needs (level l has ceil(kLsqMaxGrid / 8^(l+1)) groups).
#ifndef MPA_LSQ_FANIN
#define MPA_LSQ_FANIN 8  // (a measurement library may be built with another: make DEFS=-DMPA_LSQ_FANIN=16)
#endif
constexpr int kLsqFanIn = MPA_LSQ_FANIN;
static_assert(kLsqFanIn >= 4 && kLsqFanIn <= 16, "tree fan-in");
constexpr int kLsqMaxGrid = 1024;
constexpr int kLsqCtrPerTask = 160;  // 128 + 16 + 2 + 1, rounded up

// Several workers dispatched by the same flush run as ONE launch: workgroups
// [block0[t], block0[t+1]) belong to task t.  All tasks share (dtype, cols_pad).
constexpr int kMaxLsqTasks = 16;
constexpr int kHeadPrearmed = 4;
constexpr uint32_t kHeadCancel = 0x80000000u;
constexpr unsigned long long kPreCancel = 1ull << 63;
constexpr unsigned long long kPreSame = 1ull << 62;  // the step's arguments are `ep` as launched
struct LsqBatch {
  int ntasks;
  // 1: the process serves this one worker only (the node's placement at N = 8), so the launch
  // never shares the GPU with another task launch of its own: a lone 2048-column fp32 task then
  // takes the batched launch's 32 KiB tile (c3n8 0.76 -> 0.88 of HBM, profiles/r06_pergpu.txt)
  int alone;
  unsigned* err;
  unsigned long long spin_ticks;
  int block0[kMaxLsqTasks + 1];
  LsqTask t[kMaxLsqTasks];
  // Fused tail (the native descent loop at integer nwait == n): the task of
  // this launch that completes LAST runs the NEXT epoch's coordinator step `ep` (harvest
  // copies of this launch's replies, the iterate update, the dispatch copies of the next
  // launch's messages) in its last workgroup, so the descent loop's epoch is one launch.
  // tail: 0 none, 1 scalar elements, 2 16-B vectors.  On rank 0 of a multi-process comm the
  // epoch also has workers served by other processes: the tail first waits for their
  // completion words (tail_word[k] >= tail_target[k], bounded: err bit 32), harvests their
  // replies from its inboxes, writes their next messages over xGMI and rings their doorbells
  // (ep.door), in place of wait_words_kernel + epoch_kernel.
  int tail;
  uint32_t* tail_ctr;  // task completions of this launch (the last one resets it)
  int tail_nwait;
  const unsigned long long* tail_word[kMaxEpochChunks];
  unsigned long long tail_target[kMaxEpochChunks];
  // Fused head (the native descent loop at any nwait, every worker of the pool in this launch):
  // workgroup 0 first runs THIS epoch's coordinator step `ep` (the harvest copies of the
  // replies the call received, the iterate update, the dispatch copies of this launch's
  // messages) and publishes head_token in *head_word; every other workgroup waits for it
  // before it reads its message.  Workgroups are dispatched in order, so workgroup 0 runs
  // whatever else is resident; the wait is bounded (err bit 128).  head: 0 none, 1 / 2 as
  // tail; a launch carries a head or a tail, never both.
  //   head | kHeadPrearmed: a PRE-ARMED launch, enqueued one epoch early (transport_hip.cpp,
  //   maybe_prearm): workgroup 0 first waits for the host to decide the epoch -- *pre_go (a
  //   host-pinned word) reaching pre_token -- and reads the step's EpochArgs from *pre_ep (the
  //   same pinned mailbox) instead of `ep` -- or, go = pre_token | kPreSame, the `ep` it was
  //   launched with (the host's prediction held: no mailbox read over the bus); pre_token |
  //   kPreCancel cancels the launch (every
  //   workgroup returns, nothing is published).  Bounded like the other waits (err bit 128).
  int head;
  uint32_t* head_word;
  uint32_t head_token;  // below kHeadCancel; head_token | kHeadCancel: the launch was cancelled
  const unsigned long long* pre_go;
  const EpochArgs* pre_ep;
  unsigned long long pre_token;
  EpochArgs ep;
};
static_assert(sizeof(LsqBatch) <= 4096, "LsqBatch is passed by value as kernel arguments (4 KiB)");
// A batch with a device-armed task launches the kernel variant whose workgroups wait on the
// doorbell first; every other launch runs a variant without that prologue (its mere presence
// cost the c2 launch 19 %: profiles/r03_cross_tail.txt)
template <class Batch>
inline bool batch_armed(const Batch& b) {
  for (int k = 0; k < b.ntasks; ++k)
    if (b.t[k].door) return true;
  return false;
}
// Returns hipErrorInvalidValue if no kernel variant covers (dtype, cols).  cols > 2048 runs
// the wide two passes (launch_lsqw).
hipError_t launch_lsq(int dtype, int cols, const LsqBatch& a, hipStream_t s);
hipError_t launch_lsqw(int dtype, const LsqBatch& a, hipStream_t s);
const char* lsq_variant_name();  // the c2-shape kernel variant in use (MPA_LSQ_VARIANT)
int lsq_set_variant(int i);      // returns the number of variants, or -1 if i is out of range
// Shape helpers for the launcher's variant table.
int lsq_cols_pad(int dtype, int cols);  // 0 if unsupported
int lsq_rows_per_wave_iter(int dtype, int cols);

// One worker task of the batched multi-iterate variant (lsqb_kernel.hip):
// G = A^T (A X - B), A rows x cols bf16 (lda), X cols x 64 bf16 (the message, row-major),
// B rows x 64 bf16, G cols x 64 fp32 (the reply, row-major).
constexpr int kLsqbIterates = 64;
constexpr int kLsqbMaxSlices = 16;  // 256-column slices: cols <= 4096
constexpr int kLsqbSplitKCols = 2048;  // pass 1 holds X in registers up to this many columns
constexpr int kLsqbSplitKRows = 16;    // rows per split-K pass-1 block
struct LsqbTask {
  const void* A;
  const void* B;
  const void* X;
  void* out;
  void* R;      // [rows_pad/8][64][hi 8 | lo 8] bf16 residual (pass 1 -> pass 2)
  void* slab;   // [nrange][nslice][64 x 256] fp32 partials of pass 2
  uint32_t* ctr;  // [kLsqbMaxSlices] per-slice arrivals + [1] per-task slice completions
  unsigned long long* flag;
  unsigned long long* flag2;  // N > 1, a worker process's task: rank 0's device copy of the done word, or null
  unsigned long long seq;
  int64_t rows, lda;
  int cols;
  int grid1;           // pass-1 workgroups (256 rows each, grid-strided)
  int nrange, nslice;  // pass-2 grid = nrange * nslice
  uint32_t sbase, tbase;  // ctr values before this launch (every slice counter moves alike)
  const unsigned long long* go;  // as LsqTask::go
  const unsigned long long* door;  // as LsqTask::door
};
struct LsqbBatch {
  int ntasks;
  int splitk;  // pass 1 = the whole-row split-K kernel (every task cols <= kLsqbSplitKCols)
  unsigned* err;
  unsigned long long spin_ticks;
  int block1[kMaxLsqTasks + 1];
  int block2[kMaxLsqTasks + 1];
  LsqbTask t[kMaxLsqTasks];
};
// pass 1 + pass 2 of every task of the batch, two launches on `s`
hipError_t launch_lsqb(const LsqbBatch& a, hipStream_t s);

// Single pass by iterate halves (lsqp_kernel.hip, the c5 default for cols <= 2048): pairs of
// workgroups stream the same rows, member h owning iterates 32h .. 32h + 31 of R and G; no
// exchange between members.  Pairs [grp0[t], grp0[t+1]) serve task t (grid = 16 x ceil(pairs
// / 8): the members of pair p are blocks 16 (p / 8) + p % 8 and that + 8).
constexpr int kLsqpMaxGroups = 128;   // pairs (row groups) per task
constexpr int kLsqpCtrPerSlice = 64;  // tree counters per (half, wave): 32 + 8 + 2 + 1, rounded up
constexpr int kLsqpMaxCols = 2048;    // 8 waves x 256 columns
struct LsqpTask {
  const void* A;
  const void* B;
  const void* X;
  void* out;
  void* slab;      // [2][kLsqpMaxGroups][8 waves][32 KiB] fp32 G partials (tree reduced in place)
  uint32_t* ctr;   // [2 halves][8 waves][kLsqpCtrPerSlice] tree counters + [1] slice completions;
                   // every counter is reset by its last arriver
  unsigned long long* flag;
  unsigned long long* flag2;  // N > 1, a worker process's task: rank 0's device copy of the done word, or null
  unsigned long long seq;
  int64_t rows, lda;
  int cols;
  const unsigned long long* go;  // as LsqTask::go
  const unsigned long long* door;  // as LsqTask::door
  // column pairs (lsqc_kernel.hip) only
  unsigned long long* xg;  // [kLsqpMaxGroups][2][kLsqcXR][4][64][4] {tag, fp32} exchange granules
  int parts;               // members per row group: 2 if cols > kLsqcMemberCols, else 1
  int pub_local;  // as LsqTask::pub_local (lsqp4)
};
struct LsqpBatch {
  int ntasks;
  int pfd;  // L2 prefetch lead over the LDS-DMA, in blocks (0: none); MPA_LSQP_PF.  lsqc: phase-1 lookahead (1, 2)
  int dbg;  // measurement build only (MPA_LSQP_DBG): 1 no DMA, 2 no compute, 8/16/32 no phase 1 / reduce / phase 2
  int xred;  // lsqp4: G over the row groups in a second launch (set by launch_lsqp4; MPA_LSQP4_XRED=0: in-kernel tree)
  int grp0[kMaxLsqTasks + 1];  // lsqp/lsqp4: pairs before task t; lsqc: workgroups before task t
  LsqpTask t[kMaxLsqTasks];
  // column pairs (lsqc_kernel.hip) only
  uint32_t* tick;  // workgroup ticket counter (zero between launches: the last taker resets it)
  // bounded in-kernel waits (lsqc's exchange, a device-armed task's doorbell): error word, bound
  unsigned* err;
  unsigned long long spin_ticks;
};
hipError_t launch_lsqp(const LsqpBatch& a, hipStream_t s);
// the same batch by the one-wave-per-SIMD cut (lsqp4_kernel.hip, the default)
hipError_t launch_lsqp4(const LsqpBatch& a, hipStream_t s);
// (rounds 4-5 measured three more restructurings of lsqp4 -- phase 2 as 32x32x16 MFMAs, the
// block-pipelined kernel, the pair step -- parity-green and level with it on HBM; removed in round
// 6, their record is DESIGN.md §10 and profiles/r04_c5_*, r05_c5_pairstep.txt)
// Single pass by COLUMN pairs (lsqc_kernel.hip): the two members of a row group split the
// columns (member h: columns 1024 h .. 1024 h + 1023), each holding all 64 iterates of its G
// columns, and exchange their 16 x 64 partial products per 16-row block as tagged granules.
// Pairs form from a ticket taken at start (members only wait for running workgroups).
constexpr int kLsqcMemberCols = 1024;
constexpr int kLsqcXR = 8;           // exchange ring slots per member
constexpr int kLsqcMaxBlocks = 65535;  // 16-row blocks per row group (16-bit block field of the tag)
hipError_t launch_lsqc(const LsqpBatch& a, hipStream_t s);

// Single-pass variant (lsqf_kernel.hip): groups of P = ceil(cols / kLsqfSlice) workgroups,
// one 512-column slice each, exchanging per-block partial residuals through `xbuf`.
constexpr int kLsqfSlice = 512;
constexpr int kLsqfMaxP = 4;         // cols <= 2048
constexpr int kLsqfXR = 16;          // exchange ring slots per group
constexpr int kLsqfMaxGroups = 64;   // per task
struct LsqfTask {
  const void* A;
  const void* B;
  const void* X;
  void* out;
  void* xbuf;                  // [groups][kLsqfXR][P][4][64] f32x4 partial tiles
  unsigned long long* xflag;   // [groups][kLsqfXR][P]: (seq << 32) | (block + 1)
  void* slab;                  // [groups][P][128 KiB] G partials
  uint32_t* ctr;               // [kLsqfMaxP] per-slice group arrivals + [1] slice completions
  unsigned long long* flag;
  unsigned long long seq;
  int64_t rows, lda;
  int cols;
  uint32_t sbase, tbase;       // ctr values before this launch
  const unsigned long long* go;
};
struct LsqfBatch {
  int ntasks;
  int P;                       // members per group (every task of a batch alike)
  unsigned* err;
  unsigned long long spin_ticks;
  unsigned long long* tick;    // [8] per-XCD tickets, [8] arrivals: (tag << 32) | count
  uint32_t tag;                // this launch's tag (low half of task 0's seq)
  int lag;                     // phase 1 runs this many blocks ahead (MPA_LSQF_LAG, 1-4)
  int dbg;                     // MPA_LSQF_DBG: mode 3 loader only, 4 no exchange, 7 all groups cross-XCD; +16 wait profile
  int grp0[kMaxLsqTasks + 1];  // groups [grp0[t], grp0[t+1]) serve task t
  LsqfTask t[kMaxLsqTasks];
};
hipError_t launch_lsqf(const LsqfBatch& a, hipStream_t s);

// Single pass by iterate quarters (lsqq_kernel.hip): quads of workgroups, member q owns
// iterates 16q..16q+15 of G for all columns (cols <= 2048); no exchange between members.
struct LsqqTask {
  const void* A;
  const void* B;
  const void* X;
  void* out;
  void* slab;                  // [groups][4][ceil(cols/256)][16][64] f32x4 G partials
  uint32_t* ctr;               // [4] per-member group arrivals, [4] member completions (self-resetting)
  unsigned long long* flag;
  unsigned long long seq;
  int64_t rows, lda;
  int cols;
  const unsigned long long* go;
};
struct LsqqBatch {
  int ntasks;
  int dbg;                     // MPA_LSQQ_DBG timing probes (lsqq_kernel.hip)
  int grp0[kMaxLsqTasks + 1];  // quads [grp0[t], grp0[t+1]) serve task t; grid = 4 x quads
  LsqqTask t[kMaxLsqTasks];
};
hipError_t launch_lsqq(const LsqqBatch& a, hipStream_t s);
size_t lsqf_lds_bytes();
void lsqf_prof_dump();  // MPA_LSQF_DBG & 16: wait-cycle breakdown to stderr
void head_stamp_reset();  // MPA_HEAD_STAMP=1 (measurement build): the fused-head launch stamps
void head_stamp_dump();
void lsqp4_clock_dump();  // MPA_LSQP4_CLOCK=1: lsqp4's in-kernel clock of its last launch to stderr
void lsq_stamp_dump();    // MPA_LSQ_STAMP=1: lsq_grad_kernel's last launch timeline to stderr

struct KmapArgs {
  int kind;
  double rank;
  const uint8_t* x;
  uint64_t sl;
  uint8_t* out;
  uint64_t rl;
  Publish pub;
  // task trace (host-pinned, may be null): [0] s_memrealtime at the kernel's start, [1] just
  // before its completion store
  unsigned long long* stamp;
  int pub_local;  // as LsqTask::pub_local
};
// one wave stores s_memrealtime into *out (host-pinned): the task trace's clock calibration
hipError_t launch_clock_probe(unsigned long long* out, hipStream_t s);
hipError_t launch_kmap(const KmapArgs& a, hipStream_t s);
// one wave that waits for a device-armed task's doorbell (seq, with or without kCancelBit;
// bounded by spin_ticks: on timeout it stores seq into `cancel`, the queued task's go word, so
// the task cancels itself, and sets err bit 64), then -- a delayed worker, not cancelled -- sleeps
// delay_ticks from the ring, then acquires at system scope; the task runs behind it
hipError_t launch_door_wait(const unsigned long long* door, unsigned long long seq, unsigned long long spin_ticks,
                            unsigned* err, unsigned long long* cancel, unsigned long long delay_ticks, hipStream_t s);
// one wave that waits until s_memrealtime reaches `deadline` (a delayed worker's sleep, ahead of
// its task on its stream), at most `bound` ticks (then err bit 256)
hipError_t launch_deadline(unsigned long long deadline, unsigned long long bound, unsigned* err, hipStream_t s);
// a worker process moves its device doorbell word (a device-armed task's cancel / restore,
// hip_server.cpp disarm_all): *door = desired if it holds expect; the value it held goes to
// *old_out (host-pinned)
hipError_t launch_door_cas(unsigned long long* door, unsigned long long expect, unsigned long long desired,
                           unsigned long long* old_out, hipStream_t s);


constexpr int kMaxAggregate = 256;
struct AggregateArgs {
  const void* chunks;
  void* out;     // aggregate: out = sum w_i c_i ; update: out (= x) -= eta * sum w_i c_i
  int64_t n, elems, stride;
  double eta;
  int update;
  uint16_t* mirror;  // update only: bf16 copy of the updated fp32 out (the batched variant's X)
  double w[kMaxAggregate];
};
hipError_t launch_aggregate(int dtype, const AggregateArgs& a, hipStream_t s);

// grid (blocks) the launch uses: the caller advances the doorbell ticket by it
int epoch_grid(int dtype, const EpochArgs& a);
// the step can use 16-B vectors (element count and every pointer allow it)
bool epoch_vec(int dtype, const EpochArgs& a);
int epoch_width(int dtype, const EpochArgs& a);  // elements per thread: 1, 2 / 4 (16-B vectors), 8 (bf16 messages)
hipError_t launch_epoch(int dtype, const EpochArgs& a, hipStream_t s);

// streaming read of `bytes` (a multiple of 16) for the measured HBM read ceiling; `sink`
// holds `grid` words
hipError_t launch_read_peak(const void* p, uint64_t bytes, int grid, uint32_t* sink, hipStream_t s);
hipError_t launch_generate(void* out, int dtype, uint64_t seed, uint32_t stream, uint64_t e0, int64_t count,
                           double scale, hipStream_t s);

}  // namespace mpa
