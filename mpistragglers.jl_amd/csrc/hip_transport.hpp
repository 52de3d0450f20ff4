// The HIP transport's shared declarations: the HipComm class (a Comm whose workers are
// device tasks), its worker records, the exchange-kernel builder and the process-wide stream
// pool.  The class is implemented in three units:
//   transport_hip.cpp  the coordinator: the per-call protocol of the state machine, the
//                      native descent loop's epoch step (launch-ahead, fused tail), the gate
//   hip_server.cpp     worker processes (N > 1): doorbell serving, pre-armed tasks, HIP IPC
//   hip_launch.cpp     task launches: batching, kernel arguments, straggler timer, timing
// See transport_hip.cpp for the mapping onto the reference's MPI verbs.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "comm.hpp"
#include "kernels.hpp"
#include "shm.hpp"

#ifndef MPA_MEASURE
#define MPA_MEASURE 0
#endif

namespace mpa {

#define HIPCHECK(expr)                                                                  \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) fail(MPA_DEVICE_ERROR, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

extern int g_lsq_grid;  // mpa_tune("lsq_grid", G): workgroups per least-squares launch (0 = default)
// A/B switches of the measurement build only (make MEASURE=1): the product reads none of
// them, so the shipped behaviour cannot be switched off by an environment variable
inline const char* measure_env(const char* name) { return MPA_MEASURE ? std::getenv(name) : nullptr; }
// rank 0 waits for remote completions of a launched-ahead epoch with one wait_words_kernel
// (default) or, MPA_WAIT_VALUE_OPS=1, one hipStreamWaitValue64 per remote worker (round 1)
extern const bool g_wait_value_ops;

using Clock = std::chrono::steady_clock;

// workgroups per least-squares launch: 192 (24 per XCD, 3/4 of the CUs) streams the c2
// batch at 7.1-7.2 TB/s against 6.7-6.8 at 512 and 7.0 at 256 (profiles/r01_tune_sweep4_grid.jsonl,
// same-box bench A/B in profiles/r01_lsq_grid_ab.txt: c2 +6-7 %, c3/c4 unchanged); the read
// probe (mpa_read_bandwidth) shows the same shape: fewer, longer streams read faster
constexpr int kDefaultLaunchGrid = 192;
constexpr int kWideResidGrid = 1024;  // wide rows: pass-1 workgroups per launch (a wave per row)
constexpr int kSlabGridCap = kLsqMaxGrid;  // most workgroups a single task may be given
constexpr int kLaunchStreams = 2;
constexpr uint64_t kTimerSpinNs = 1000000;
// A delayed task's own overhead (launch -> completion word seen, ~30-40 us: the median latency
// deviation of the gated replays, profiles/r04_gated_stall.txt) comes out of its sleep.
constexpr int64_t kDelayLeadNs = 35000;  // the straggler timer spins the last 1 ms before a due launch
constexpr uint64_t kTimerPauseNs = 50000;  // ... yielding the core until the last 50 us, then pause-spinning
// A device-deadline delay (deadline_kernel already queued ahead of the task): what remains after
// the deadline is the task's dispatch behind it, the task itself and its completion word
// crossing the bus (MPA_DEADLINE_LEAD_NS overrides it)
constexpr int64_t kDeadlineLeadNs = 8000;
// the host <-> device clock map behind device deadlines is refreshed this often by a sampling
// thread of its own (one probe round trip on a stream of its own: never on the coordinator's
// path -- a probe taken inside a call cost kmap2_n9 a 1.4 ms harvest hop, r06d), a sample with a
// longer round trip is dropped, and the rate is measured over at least kClockRateSpanNs
constexpr uint64_t kClockRecalNs = 250000000;
constexpr int64_t kClockMaxRttNs = 40000;
constexpr int64_t kClockRateSpanNs = 1000000000;
// batched multi-iterate task: pass-1 / pass-2 workgroups per launch (= resident: 1 x 512 /
// 2 x 256 threads per CU by VGPRs), and the most row ranges a pass-2 task is split into
constexpr int kLsqbGrid1 = 512;  // two 8-wave workgroups per CU: pass 1 4.74-4.88 -> 5.11 TB/s (profiles/r01_lsqb_grid.txt)
constexpr int kLsqbGrid2 = 512;
constexpr int kLsqbRangeCap = 128;
constexpr int kLsqfGrid = 256;  // single-pass batched launch: one 768-thread workgroup per CU
constexpr size_t kLsqfCtrBytes = 64 + 16 * sizeof(unsigned long long);

inline bool env_off(const char* name) {
  const char* e = std::getenv(name);
  return e && *e == '0';
}

// c5 launch grids (MPA_LSQB_GRID1 / MPA_LSQB_GRID2 override them for measurement)
inline int lsqb_grid(int pass) {
  static const int g1 = [] { const char* e = measure_env("MPA_LSQB_GRID1"); return e ? std::max(8, std::atoi(e)) : kLsqbGrid1; }();
  static const int g2 = [] { const char* e = measure_env("MPA_LSQB_GRID2"); return e ? std::max(8, std::atoi(e)) : kLsqbGrid2; }();
  return pass == 1 ? g1 : g2;
}

// Process-wide, capped set of CU-masked streams (hip_launch.cpp): communicators come and go
// (tests create many), but the HSA queues behind their streams are a bounded hardware
// resource (past ~20 per device the scheduler time-slices them and launches stall up to
// ~10 ms), so a destroyed comm returns its streams and the next comm reuses them; past the
// cap (MPA_MAX_QUEUES) streams are shared.
constexpr int kDefaultMaxQueues = 10;  // 12 until round 5; the comm's own coordinator stream is one of them
enum class StreamKind { kWorker, kLaunch, kCoord };
// reserved: the stream leaves CU 0 of every XCD (CU-mask bits 0-7, tools/probe_cumask.hip:
// bit b is CU b / 8 of XCD b % 8) to the coordinator's own stream (DESIGN.md §5, N > 1)
hipStream_t make_queue_stream(int device, StreamKind kind, bool reserved = false);
constexpr int kReservedCus = 8;
void release_queue_stream(int device, hipStream_t s);
bool stream_shared(hipStream_t s);  // more than one worker / comm launches on it
int queue_streams(int device);      // CU-masked streams the process holds on the device
int queues_past_cap();             // queues created past the cap (a stream kind that had none)

struct HipWorker {
  bool here = true;     // its tasks run in this process
  bool remote = false;  // coordinator's view of a worker served by another process
  hipStream_t stream = nullptr;
  unsigned long long seq = 0;  // coordinator: tasks posted; server: tasks served
  void* slab = nullptr;
  int slab_grid = 0;
  size_t slab_bytes = 0;
  uint32_t* wctr = nullptr;  // wide rows (lsqw_kernel.hip): per-slice tree + completion counters
  // batched multi-iterate task (lsqb_kernel.hip): residual scratch, pass-2 partials,
  // counters and their running totals
  void* lsqb_R = nullptr;
  size_t lsqb_R_bytes = 0;
  void* lsqb_slab = nullptr;
  size_t lsqb_slab_bytes = 0;
  uint32_t* lsqb_ctr = nullptr;
  uint32_t lsqb_sbase = 0, lsqb_tbase = 0;
  // single-pass variant (lsqf_kernel.hip): exchange ring, its flags, counters
  // ([kLsqfMaxP] slices, [1] completions, [1] group tickets) and their running totals
  void* lsqf_x = nullptr;
  unsigned long long* lsqf_flag = nullptr;
  uint32_t* lsqf_ctr = nullptr;
  uint32_t* lsqq_ctr = nullptr;  // quad kernel: [4] member arrivals, [4] completions (self-resetting)
  // pair single pass (lsqp_kernel.hip): G partials and tree counters (self-resetting)
  void* lsqp_slab = nullptr;
  uint32_t* lsqp_ctr = nullptr;  // [2][8][kLsqpCtrPerSlice] tree, [1] completions, then the lsqc ticket
  unsigned long long* lsqc_xg = nullptr;  // column pairs: exchange granules
  uint32_t lsqf_sbase = 0, lsqf_tbase = 0;
  // current task
  int64_t slot = -1;
  const uint8_t* x = nullptr;
  uint8_t* out = nullptr;
  size_t sl = 0, rl = 0;
  unsigned long long* flag_host = nullptr;  // completion word, host view
  unsigned long long* flag_dev = nullptr;   // the same word, device view
  // mailbox (remote worker on the coordinator / served worker in a worker process)
  BoxHeader* box = nullptr;
  uint8_t* box_msg_dev = nullptr;
  uint8_t* box_reply_dev = nullptr;
  unsigned long long* box_door_dev = nullptr;
  uint8_t* xslot = nullptr;  // server: the worker's device message slot
  // device-memory (xGMI) payload path (shm.hpp kPathDevice): coordinator: the server's
  // message slot opened by IPC, and its own reply inbox; server: rank 0's inbox opened
  bool path_known = false, path_dev = false;
  uint8_t* peer_msg = nullptr;
  uint8_t* reply_inbox = nullptr;
  uint8_t* peer_reply = nullptr;
  // server, pre-armed tasks (serve()): armed = how many tasks, `seq - armed + 1` .. `seq`, are
  // queued behind their doorbells (at most arm_depth_); two cancel words (host-pinned, device
  // view), task s using word s & 1; the counter bases each armed task started from (by s & 1),
  // restored if it is cancelled
  int armed = 0;
  unsigned long long* cancel_host = nullptr;
  unsigned long long* cancel_dev = nullptr;
  // coordinator, launch-ahead: the next post / harvest of this worker is already enqueued
  bool preposted = false, preharvest = false;
  uint32_t arm_sbase[2] = {0, 0}, arm_tbase[2] = {0, 0}, arm_fsbase[2] = {0, 0}, arm_ftbase[2] = {0, 0};
  int64_t tslot = -1;  // task trace (mpa_comm_set_trace): the current task's entry, -1 none
};

// Accumulates copy items and doorbells into as few exchange launches as fit the kernel
// argument (kMaxCopies / kMaxDoorbells per launch), in order.
class ExchangeBuilder {
 public:
  ExchangeBuilder(uint32_t* ticket, uint32_t* ticket_count, hipStream_t s)
      : ticket_(ticket), count_(ticket_count), s_(s) {
    reset();
  }
  void reserve(int copies, int doors) {
    if (a_.ncopy + copies > kMaxCopies || a_.ndoor + doors > kMaxDoorbells) launch();
  }
  void copy(const uint8_t* src, uint8_t* dst, uint64_t bytes) {
    if (bytes == 0) return;
    reserve(1, 0);
    CopyItem& c = a_.c[a_.ncopy];
    c.src = src;
    c.dst = dst;
    c.bytes = bytes;
    a_.block0[a_.ncopy] = blocks_;
    blocks_ += int((bytes + kPart - 1) / kPart);
    a_.ncopy += 1;
    a_.block0[a_.ncopy] = blocks_;
  }
  void door(unsigned long long* addr, unsigned long long value) {
    reserve(0, 1);
    a_.door[a_.ndoor] = addr;
    a_.doorval[a_.ndoor] = value;
    a_.ndoor += 1;
  }
  void launch() {
    if (a_.ncopy == 0 && a_.ndoor == 0) return;
    const int grid = blocks_ > 0 ? blocks_ : 1;
    if (a_.ndoor > 0) {
      a_.ticket = ticket_;
      a_.ticket_base = *count_;
      *count_ += uint32_t(grid);
    }
    HIPCHECK(launch_exchange(a_, s_));
    reset();
  }

 private:
  static constexpr uint64_t kPart = 64 * 1024;
  void reset() {
    a_ = ExchangeArgs{};
    a_.part = kPart;
    blocks_ = 0;
  }
  ExchangeArgs a_{};
  int blocks_ = 0;
  uint32_t* ticket_;
  uint32_t* count_;
  hipStream_t s_;
};

// Host-side time per coordinator step (measurement build, MPA_HOST_PROF=1: the descent loop
// prints it): where a latency-bound epoch (c1) spends the coordinator thread's time
enum HostProfKey { kHpAsyncmap, kHpFlush, kHpPreConsume, kHpPrearm, kHpLaunch, kHpWaitany, kHpHarvest, kHpPost, kHpUpdate,
                   kHpKeys };
#if MPA_MEASURE
struct HostProf {
  std::atomic<int64_t> ns[kHpKeys];
  std::atomic<int64_t> n[kHpKeys];
};
extern HostProf g_hprof;
struct HostProfScope {
  int k;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  ~HostProfScope() {
    g_hprof.ns[k].fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count(),
                            std::memory_order_relaxed);
    g_hprof.n[k].fetch_add(1, std::memory_order_relaxed);
  }
};
#define MPA_HPROF(key) ::mpa::HostProfScope hprof_scope_{key}
// host event stamps (measurement build, MPA_HOST_STAMP=<dir>: <dir>/<pid>.txt at exit, one line per
// event: kind, two integers, CLOCK_MONOTONIC ns -- the clock rocprofv3's kernel trace reports, so a
// run's host events line up with its kernels; tools/arm_timeline.py)
void host_stamp(char kind, int64_t a, int64_t b);
#define MPA_HSTAMP(kind, a, b) ::mpa::host_stamp(kind, int64_t(a), int64_t(b))
#else
#define MPA_HPROF(key) (void)0
#define MPA_HSTAMP(kind, a, b) (void)0
#endif

class HipComm final : public Comm {
 public:
  enum Role { SOLO, COORD, SERVER };

  HipComm(int64_t n, const int* devices, const int* placement, int my_rank, ShmRegion* region);

  ~HipComm() override;

  int transport() const override { return MPA_TRANSPORT_HIP; }
  // The coordinator stream.  The legacy default stream (NULL, torch's default) is replaced by
  // the comm's own stream: HIP orders every command of the NULL stream after all the work
  // queued on the device's blocking streams, the worker streams included, so an epoch step
  // or a stale harvest on it waited for the stragglers' running tasks (c3: 0.1-0.6 ms per
  // epoch step, up to 5.7 ms per harvest; profiles/r05_null_stream.txt).  The comm's stream is
  // a blocking stream itself, so HIP still orders it with the caller's NULL-stream work both
  // ways.  MPA_OWN_COORD=0 keeps the NULL stream.
  // The caller's stream (the Python layer passes torch's current one when it changes; Julia
  // the task-local one).  The NULL stream becomes the comm's own blocking stream, which HIP
  // still orders with the caller's NULL-stream work both ways.  A change of coordinator stream
  // orders the new one after everything already queued on the old (a launch-ahead epoch, a
  // pre-armed head): ADVICE r05.  Work the caller queues on OTHER streams is the caller's to
  // order (torch: wait_stream on the current stream), as for any kernel library.
  void set_stream(hipStream_t s) {
    caller_null_ = s == nullptr || s == hipStreamLegacy;
    hipStream_t next = caller_null_ && own_coord_ ? own_coord_ : s;
    if (next != coord_) {
      HIPCHECK(hipEventRecord(switch_ev_, coord_));
      HIPCHECK(hipStreamWaitEvent(next, switch_ev_, 0));
    }
    coord_ = next;
  }
  hipStream_t stream() const { return coord_; }

  void begin_call(const CallBufs& b) override {
    if (role_ == SERVER) fail(MPA_ERROR, "asyncmap!/waitall! run on rank 0; this process serves workers (mpa_comm_serve)");
    check_buffers(b);
    b_ = b;
    call_posts_.clear();
  }
  // the call's buffers must be memory the GPU addresses (device memory, or host memory
  // registered with HIP): pageable host memory -- a host array handed to a device comm by
  // mistake -- is an ArgumentError, not a kernel fault.  Checked when the pointers change.
  void check_buffers(const CallBufs& b);

  void post(int64_t i, int64_t rank, int64_t tag) override;

  void harvest(int64_t i, int64_t rank) override;

  bool test(int64_t i, int64_t rank) override {
    (void)i;
    return done(rank);
  }

  int64_t waitany(int64_t n, const int64_t* ranks, const uint8_t* live) override;

  void waitall(int64_t n, const int64_t* ranks, const uint8_t* live) override;

  void flush() override;

  void end_call() override {
    may_hold_ = false;
    if (!defer_end_) flush();
  }

  // A stale worker's re-dispatch (pool.cpp, the wait loop): its message copies and the
  // stale harvest go out now, its task launch is HELD (undelayed least-squares tasks only)
  // and joins the next flush's batch, or is launched when a wait would block.  On one GPU
  // the coordinator stream runs launches in order, so a re-dispatch enqueued behind the
  // running batch starts when that batch ends either way; held, it runs INSIDE the next
  // epoch's batched launch instead of alone before it (c5, nwait 7 of 8: one 8-task launch
  // per epoch instead of a 1-task launch and a 7-task launch, profiles/r02_c5_hold_ab.txt).
  // The pool's state machine is unchanged; MPA_HOLD=0 launches re-dispatches at once.
  // Holding pays only where the held task has a batch to join: another local undelayed
  // least-squares worker of this process.  Rank 0 of the node's placement serves one worker, the
  // stale one itself: held, its task would only start an epoch late (r06b), so it launches at
  // once.  (Where peers exist the hold stays whether or not they are still running: c1's
  // whole-pool pre-armed launches depend on the held task joining the next one, -18 % in r06d.)
  void flush_stale() override {
    hold_next_ = hold_ok_ && has_batch_peer();
    flush();
    hold_next_ = false;
  }
  // a local undelayed least-squares worker other than the ones this flush posts
  bool has_batch_peer() const {
    for (int64_t r = 1; r <= nworkers_; ++r) {
      const HipWorker& w = w_[size_t(r - 1)];
      const TaskSpec& ts = tasks_[size_t(r - 1)];
      if (!w.here || w.remote || !ts.delays_ns.empty() || (ts.kind != MPA_TASK_LSQ && ts.kind != MPA_TASK_LSQ_BATCH))
        continue;
      if (std::find(posts_.begin(), posts_.end(), r) == posts_.end()) return true;
    }
    return false;
  }
  void set_wait_hold(bool may_hold) override { may_hold_ = may_hold; }
  void release_held();

  // ---- the native descent loop (capi.cpp descent_loop) ----
  // The iterate update between two asyncmap! calls, folded into the next flush (one epoch
  // kernel: harvests, update, dispatch copies, doorbells) instead of its own launches.
  struct UpdateSpec {
    int dtype = MPA_F32;  // of x and of the recv chunks
    int64_t elems = 0;
    std::vector<double> w;
    double eta = 0;
    void* x = nullptr;
    uint16_t* mirror = nullptr;  // bf16 copy of x; the message when msg_bf16
    bool msg_bf16 = false;
  };
  int payload_path(int64_t rank) const {
    if (rank < 1 || rank > nworkers_) return 0;
    const HipWorker& w = w_[size_t(rank - 1)];
    return w.remote && w.path_known ? (w.path_dev ? int(kPathDevice) : int(kPathHost)) : 0;
  }
  // end_call() leaves the call's harvests pending (they join the next flush's epoch kernel)
  void set_defer_end_flush(bool on, bool prearm_ok = false) {
    if (!on) cancel_pre();
    defer_end_ = on;
    prearm_loop_ = on && prearm_ok;
    if (!on) tail_next_ = tail_pending_ = head_next_ = false;  // the descent loop ended (or failed)
  }
  void stage_update(const UpdateSpec& u);
  // Launch-ahead (integer nwait == n): the call returns only once all n tasks it posts have
  // completed fresh, so the next epoch is fully determined before this call's waits begin:
  // harvest all n, update with weight 1 each, re-post all n.  The phase-2 flush of such a
  // call enqueues that next epoch (epoch kernel + tasks) right behind this one; the next
  // call then finds its posts already enqueued.  `epochs_left` = calls still to come.
  void set_ahead(int64_t epochs_left, const UpdateSpec& pred) {
    ahead_left_ = epochs_left;
    ahead_pred_ = pred;
  }

  uint64_t now_ns() override {
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count());
  }

  int64_t tasks_done(int64_t rank) override {
    return int64_t(__atomic_load_n(w_[size_t(rank - 1)].flag_host, __ATOMIC_ACQUIRE));
  }

  void shutdown() override;

  void on_task_changed(int64_t rank) override;
  void on_delays_changed(int64_t rank) override;

  // ---- worker process: watch the doorbells of the workers served here ----
  // Least-squares workers whose messages arrive in this GPU's slot are DEVICE-ARMED
  // (armable): their next task (two, arm_depth) is already queued behind a one-wave wait for
  // the worker's device doorbell, which rank 0 stores over xGMI right after the message (a
  // delayed worker's wait then sleeps its delay).  Other workers (the reference's test
  // programs, the host mailbox) are launched by this thread when it sees their shared-memory
  // doorbell.  serve() returns at pause / shutdown after disarming: the waiting tasks rank 0
  // has not rung are released with kCancelBit and return without writing or publishing.
  void serve();

  // ---- device-armed tasks (server) ----
  // MPA_ARM=2 (default): where a process serves ONE worker (N = 8); MPA_ARM=1: every eligible
  // worker; MPA_ARM=0: never.  Round 2's armed launch waited behind hipStreamWaitValue64 on
  // the host doorbell (a blit kernel per wait) and read the host go word from every lane:
  // 7-15x slower tasks (profiles/r02_arm_go_word.txt); the go word is now read once by the
  // reply's writer and the wait is the kernel's own poll of device memory (wait_door).  With
  // several workers the host-launched path batches a flush's tasks into one launch.
  bool armable(int64_t rank) const;
  // how many tasks of an armable worker stay queued behind their doorbells: 2 on a GPU that rank 0
  // does not use (the node's placement), so the task of the epoch after next is enqueued while
  // this one runs and the last worker to finish an epoch starts the next one from its doorbell,
  // not from this thread's re-arm; 1 on rank 0's GPU (MPA_ARM_DEPTH=1 / 2 overrides)
  int arm_depth(int64_t rank) const;
  // local workers that serve() arms: each armed launch gets its share of the launch grid
  int armed_share() const {
    int k = 0;
    for (int64_t r = 1; r <= nworkers_; ++r) k += w_[size_t(r - 1)].here && armable(r);
    return k > 0 ? k : 1;
  }

  // message / reply bytes of a task as armed (the post is checked against them afterwards)
  static size_t task_msg_bytes(const TaskSpec& ts) {
    return ts.kind == MPA_TASK_LSQ_BATCH ? size_t(ts.cols) * size_t(ts.k) * 2
                                         : size_t(ts.cols) * (ts.dtype == MPA_F64 ? 8 : 4);
  }

  // launch task seq+1 of `rank` on its stream, behind a wait for the device doorbell
  void arm(int64_t rank);
  // arm until arm_depth(rank) tasks are queued
  void arm_up(int64_t rank);

  // release every waiting armed task: one whose doorbell rank 0 has not rung is cancelled
  // (cancel word := its seq, then device doorbell := seq | kCancelBit to release the wait;
  // both restored once the stream has drained), one already rung completes.  A task
  // cancelled in a race with rank 0's ring did not publish: its doorbell is served by the
  // next serve() session (seq rolled back).
  void disarm_all();
  bool door_cas(const HipWorker& w, unsigned long long expect, unsigned long long desired);

  void pause_servers() {
    if (role_ != COORD) fail(MPA_ERROR, "only rank 0 of a multi-process communicator pauses its servers");
    __atomic_fetch_add(&region_->header()->gen, 1ull, __ATOMIC_RELEASE);
  }

 private:
  struct Harvest {
    int64_t slot, rank;
  };

  void add_harvest(ExchangeBuilder& xb, const Harvest& h) {
    const HipWorker& w = w_[size_t(h.rank - 1)];
    const uint8_t* src = w.remote ? reply_src(w) : b_.irecvbuf + size_t(h.slot) * b_.rl;
    xb.copy(src, b_.recvbuf + size_t(h.slot) * b_.rl, b_.rl);
  }

  // tasks of the workers served here among `posted`, behind the exchange / epoch kernel
  void launch_local(const std::vector<int64_t>& posted);

  // the update as its own launch (the unfused path)
  void launch_update(const UpdateSpec& u);

  bool fused_ok(const UpdateSpec& u, const std::vector<int64_t>& posted) const;

  // the epoch step can ride as the fused tail of the launch of `posted`: one batched
  // least-squares launch on the coordinator stream (local, undelayed, same shape, the
  // update's dtype), no doorbells, no bf16 mirror
  bool tail_fits(const std::vector<int64_t>& posted, const UpdateSpec& u) const;

  // ONE epoch kernel: harvests [0, before) of `hv`, the update, harvests [before, end), the
  // dispatch copies of the posts (isendbuf slot; mailbox + doorbell for a remote worker)
  void emit_epoch(const std::vector<Harvest>& hv, size_t before, const std::vector<int64_t>& posted,
                  const UpdateSpec& u, hipStream_t s);

  // the arguments of one epoch step (no doorbell ticket yet)
  EpochArgs epoch_args(const std::vector<Harvest>& hv, size_t before, const std::vector<int64_t>& posted,
                       const UpdateSpec& u) const;

  // enqueue the next epoch of an await-all call (set_ahead), once per call, when this
  // call has posted every worker of the pool
  void maybe_ahead();

  // ---- device-memory (xGMI) payload path (shm.hpp kPathDevice) ----
  // A fine-grained device buffer exported by a HIP IPC handle into `handle`; `state` tells
  // the other process whether it may open it.  Falls back to a plain allocation (state
  // kIpcFailed, payloads then go through the host mailbox) if fine-grained memory or IPC is
  // unavailable, or with MPA_XGMI=0.
  void* ipc_alloc(size_t bytes, char* handle, volatile uint32_t* state);

  void* ipc_open(const char* handle, int peer_dev);

  // coordinator, first post to a remote worker: once the server has exported its message
  // slot and opened our reply inbox, open its slot and fix the path for good
  void decide_path(int64_t rank);

  // server: open rank 0's reply inbox once it is exported; true once rank 0 fixed the path
  bool server_path(int64_t rank);

  // where rank 0 stores a remote worker's message / reads its reply
  uint8_t* msg_dst(const HipWorker& w) const { return w.path_dev ? w.peer_msg : w.box_msg_dev; }
  const uint8_t* reply_src(const HipWorker& w) const { return w.path_dev ? w.reply_inbox : w.box_reply_dev; }
  // where a served worker's task writes its reply
  uint8_t* reply_dst(const HipWorker& w) const { return w.path_dev ? w.peer_reply : w.box_reply_dev; }
  // the worker's device doorbell word, after the message in its fine-grained slot (server:
  // its own slot; rank 0: the slot opened by IPC, device path only)
  size_t door_off() const { return (region_->max_msg() + 255) / 256 * 256; }
  unsigned long long* peer_door(const HipWorker& w) const {
    return reinterpret_cast<unsigned long long*>(w.peer_msg + door_off());
  }
  unsigned long long* own_door(const HipWorker& w) const {
    return reinterpret_cast<unsigned long long*>(w.xslot + door_off());
  }

  bool done(int64_t rank) const {
    const HipWorker& w = w_[size_t(rank - 1)];
    return __atomic_load_n(w.flag_host, __ATOMIC_ACQUIRE) >= w.seq && gate_open(rank, w.seq);
  }

  int64_t counter(const char* name) const override;

  // gated replay hooks (gate.cpp): the coordinator's view of its workers
  bool gate_supported() const override { return role_ != SERVER; }
  uint64_t gate_posted(int64_t rank) override { return w_[size_t(rank - 1)].seq; }
  uint64_t gate_finished(int64_t rank) override { return __atomic_load_n(w_[size_t(rank - 1)].flag_host, __ATOMIC_ACQUIRE); }
  void gate_launch(int64_t rank) override {
    // a held re-dispatch the schedule completes: launch it (with the rest of the held batch)
    if (std::find(held_.begin(), held_.end(), rank) != held_.end()) release_held();
  }
  void gate_poll(double waited_s) override {
    watchdog(Clock::now(), /*timeout=*/false);
    if (timeout_s_ > 0 && waited_s > timeout_s_)
      fail(MPA_DEVICE_ERROR, "gated replay: waited more than %.0f s for a released task (MPA_WAIT_TIMEOUT_S)", timeout_s_);
  }

  unsigned device_error() const {
    unsigned e = __atomic_load_n(err_, __ATOMIC_ACQUIRE);
    if (region_) e |= __atomic_load_n(&region_->header()->err, __ATOMIC_ACQUIRE);
    return e;
  }

  void watchdog(Clock::time_point t0, bool timeout = true);

  static void check_stream(hipStream_t s) {
    const hipError_t q = hipStreamQuery(s);
    if (q != hipSuccess && q != hipErrorNotReady) fail(MPA_DEVICE_ERROR, "worker stream error: %s", hipGetErrorString(q));
  }

  void check_task(int64_t rank, const TaskSpec& ts, size_t sl, size_t rl);

  void prepare_lsq(int64_t rank, const TaskSpec& ts);

  // batched multi-iterate task: validate, size the residual scratch / partial slab
  void prepare_lsqb(int64_t rank, const TaskSpec& ts);

  // workgroups per task in a least-squares launch of `ntasks` tasks
  int lsq_grid(const TaskSpec& ts, const HipWorker& w, int ntasks) const;

  // Tasks of one flush (coordinator) or one doorbell scan (server).  Least-squares tasks
  // without an injected delay run as ONE batched launch (per kernel variant, <=
  // kMaxLsqTasks each) on an idle launch stream; a task with a delay runs on its worker's
  // own stream behind a delay kernel, so a straggler never holds back another worker;
  // reference-test tasks (kmap/echo) run per worker.  `staged`: the message sits in a
  // mailbox and is first copied into the worker's device slot on the launch's stream.
  void launch_tasks(const std::vector<int64_t>& ranks, bool staged, bool on_coord = false);

  // ---- straggler emulation -------------------------------------------------------------
  // A worker with a delay schedule sleeps `delay` ns after its message is delivered and
  // then computes (the reference worker's `sleep(rand())` before its reply,
  // examples/iterative_example.jl:74).  Default: a host timer thread launches the task kernel
  // when it is due, so a sleeping worker has nothing queued on the GPU.  MPA_DELAY=device: a
  // one-wave sleep kernel queued ahead of the task on the worker's stream instead -- exact on
  // the device clock, but CU-masked streams are blocking streams, so every operation a
  // caller issues on the legacy NULL stream then waits for every sleeping straggler
  // (profiles/r04_delay_on_device.txt).  Round 3's ~20 ms outliers were the process's queue
  // count, not the timer (profiles/r04_gated_stall.txt).
  static uint64_t mono_ns() {
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count());
  }

  struct Deferred {
    uint64_t due;
    std::function<void()> go;
    bool operator<(const Deferred& o) const { return due > o.due; }  // min-heap on due
  };

  void defer(uint64_t due, std::function<void()> go);

  void timer_loop();

  // every deferred launch issued (shutdown)
  void drain_deferred() {
    std::unique_lock<std::mutex> lk(tmu_);
    if (!timer_.joinable()) return;
    tidle_.wait(lk, [this]() { return (deferred_.empty() && !tbusy_) || tstop_; });
  }

  // pending launches are dropped (the comm is being destroyed)
  void stop_timer();

  void check_timer();

  void stage_in(const std::vector<int64_t>& ranks, hipStream_t s);

  // MPA_DEBUG=1: pointer attributes of everything handed to a kernel
  static void describe(const char* what, const void* p);

  unsigned long long spin_ticks() const { return (unsigned long long)(timeout_s_ * rt_hz_); }

  // the worker's own stream (delayed tasks, pre-armed tasks), created on first use
  hipStream_t worker_stream(HipWorker& w) {
    if (!w.stream) w.stream = make_queue_stream(dev_, StreamKind::kWorker, reserve_cus_);
    return w.stream;
  }
  // launch stream k (created on first use, up to kLaunchStreams)
  hipStream_t launch_stream(size_t k) {
    while (launch_streams_.size() <= k) launch_streams_.push_back(make_queue_stream(dev_, StreamKind::kLaunch, reserve_cus_));
    return launch_streams_[k];
  }

  // a launch stream with no pending work (so a batch never queues behind an unrelated
  // straggler's kernel); round-robin if every one is busy; a new one while fewer than
  // kLaunchStreams exist and all are busy
  hipStream_t pick_launch_stream();

  void launch_lsq_batch(const std::vector<int64_t>& ranks, int dtype, hipStream_t s);

  // kernel arguments of one launch over `ranks`
  // `share`: the launch grid is divided as if this many tasks ran at once (concurrent
  // single-task launches of pre-armed workers)
  LsqBatch build_lsq_batch(const std::vector<int64_t>& ranks, int dtype, double* bytes_out, int share = 0);

  void launch_lsqb_batch(const std::vector<int64_t>& ranks, hipStream_t s) {
    double bytes = 0;
    const LsqbLaunch b = build_lsqb_batch(ranks, &bytes);
    enqueue_lsqb(b, s, bytes);
  }

  // A batched multi-iterate launch: the single-pass kernel (lsqf_kernel.hip) where every
  // task of the batch has the same slice count (cols <= 2048) and MPA_LSQF is not 0, else
  // the two passes (lsqb_kernel.hip).
  struct LsqbLaunch {
    bool pair = false;   // lsqp (the default single pass)
    bool pair8 = false;  // ... by the eight-wave cut (MPA_LSQP=8)
    bool cpair = false;  // ... by column pairs (lsqc_kernel.hip)
    bool fused = false;  // lsqf (opt-in)
    bool quad = false;   // lsqq
    LsqbBatch two{};
    LsqfBatch one{};
    LsqqBatch four{};
    LsqpBatch halves{};
    void set_go(const unsigned long long* go) {
      if (pair) halves.t[0].go = go;
      else if (quad) four.t[0].go = go;
      else if (fused) one.t[0].go = go;
      else two.t[0].go = go;
    }
    // device-armed launches: the product's kernels (lsqp4, the two passes) only
    void set_door(const unsigned long long* door) {
      if (pair && !pair8 && !cpair) halves.t[0].door = door;
      else if (!pair && !quad && !fused) two.t[0].door = door;
      else fail(MPA_ERROR, "device-armed tasks run the product's batched kernels only");
    }
  };

  // the iterate-halves single pass (lsqp_kernel.hip): the default for cols <= 2048
  // (MPA_LSQP=0 selects the two passes)
  bool lsqp_enabled(const std::vector<int64_t>& ranks) const;

  // column pairs (lsqc_kernel.hip): a row group of a task with more than 1024 columns is a
  // pair of workgroups (one each, 1024 columns and all 64 iterates), of a narrower task one
  // workgroup; 256 workgroups (one per CU) dealt over the tasks.  Row groups of at most
  // kLsqcMaxBlocks blocks (the tag's block field), else the iterate-halves kernel stays.
  static int lsqc_parts(int64_t cols) { return cols > kLsqcMemberCols ? 2 : 1; }
  int lsqc_groups(const TaskSpec& ts, int split, int k) const;
  bool lsqc_fits(const std::vector<int64_t>& ranks, const LsqpBatch& b, int share) const;
  void build_lsqc(const std::vector<int64_t>& ranks, int share, LsqbLaunch& L);

  // the iterate-quarter single pass (lsqq_kernel.hip): cols <= 2048 on every task
  bool lsqq_enabled(const std::vector<int64_t>& ranks) const;

  bool lsqf_enabled(const std::vector<int64_t>& ranks) const;

  // kernel arguments over `ranks`; advances the workers' counter bases.  Algorithmic bytes
  // per task: A + B + X + G.
  // workers of this process with a batched least-squares task: a single-pass launch gives
  // each of its tasks the grid share of one of them, so that the launches of one epoch (all
  // fresh tasks, then a stale worker's re-dispatch, src/MPIAsyncPools.jl:177-184) run side
  // by side on disjoint CUs instead of the later one queueing behind a full-chip grid
  int lsqb_share() const;

  LsqbLaunch build_lsqb_batch(const std::vector<int64_t>& ranks, double* bytes_out, int share = 0);

  void enqueue_lsqb(const LsqbLaunch& b, hipStream_t s, double bytes, int64_t armed_rank = 0);

  // enqueue one least-squares launch on `s` (coordinator / server thread or timer thread)
  void enqueue_lsq(const LsqBatch& b, int dtype, int cols, hipStream_t s, double bytes, int64_t armed_rank = 0,
                   bool untimed = false);

 public:
  // ---- kernel timing (HIP events around every least-squares launch) ----
  // period 0 off; period k >= 1: one in every k launches of each kind is bracketed by events
  // (armed launches always are: void_timing() cancels the rank's last timed one)
  void set_timing(int period) {
    if (period <= 0) {
      reap_timing(true);
      timing_ = false;
      return;
    }
    timing_period_ = period;
    t_seq_ = 0;
    x_seq_ = 0;
    timing_ = true;
  }
  // launches, total kernel ms, total algorithmic bytes, and the ms during which at least
  // one timed launch was running (the union of their intervals: concurrent single-task
  // launches of delayed workers overlap) since the last call
  void timing(double out[4]);

 private:
  // epoch kernels timed since the last exchange_timing(): launches, ms, remote payload bytes
  struct XTimed {
    hipEvent_t start, stop;
    double remote_bytes;
  };
  std::vector<XTimed> xtimed_;
  double x_launches_ = 0, x_ms_ = 0, x_remote_ = 0;
  void reap_xtiming();

 public:
  void exchange_timing(double out[3]);

  // ---- task trace (diagnostics; mpa_comm_set_trace / mpa_comm_trace) ----
  // One entry per posted task of this process's workers, kTraceFields int64 each, host
  // steady-clock ns (0: not reached): rank, seq, post (dispatch), due (post + injected delay,
  // the oracle's completion time), call / ret (the launch call of the task kernel: entered,
  // returned -- the timer thread's for a delayed task), start / pub (the kernel's first
  // instruction and its completion store, read on the device's s_memrealtime and mapped to
  // host time by two clock calibrations), gate (the gate step that waits for it began), seen
  // (the gate observed the completion), harvest (phase 1 / wait loop took it).  Stamps are
  // written for the reference's worker programs (kmap tasks); least-squares tasks get the host
  // fields only.
  static constexpr int kTraceFields = 11;
  enum TraceField { kTRank, kTSeq, kTPost, kTDue, kTCall, kTRet, kTStart, kTPub, kTGate, kTSeen, kTHarvest };
  void set_trace(int64_t capacity);
  int64_t read_trace(int64_t* out, int64_t capacity);
  void gate_seen(int64_t rank, uint64_t seq, uint64_t step_begin_ns) override;

 private:
  int64_t* trace_ = nullptr;  // host-pinned, capacity x kTraceFields
  int64_t trace_cap_ = 0, trace_n_ = 0;
  uint64_t* clock_probe_ = nullptr;  // host-pinned word the calibration kernel stores into
  int64_t cal_ticks0_ = 0, cal_ns0_ = 0;  // (device ticks, host ns) at set_trace
  void calibrate(int64_t* ticks, int64_t* ns);
  void trace_post(HipWorker& w, int64_t rank);
  int64_t* trace_entry(const HipWorker& w) {
    return trace_ && w.tslot >= 0 ? trace_ + w.tslot * kTraceFields : nullptr;
  }

 private:
  struct TimedLaunch {
    hipEvent_t start, stop;
    double bytes;
    int64_t rank;  // pre-armed launch of this worker (0: none)
    bool void_ = false;  // cancelled before it ran: not counted
  };

  // the pending timed launch armed for `rank` was cancelled
  void void_timing(int64_t rank);

  // caller holds tm_mu_ (event_pool_ is shared with the straggler timer thread)
  hipEvent_t take_event();

  void reap_timing(bool block);

  Role role_ = SOLO;
  std::vector<HipWorker> w_;
  ShmRegion* region_ = nullptr;
  int my_rank_ = 0;
  int dev_ = 0;
  hipStream_t coord_ = nullptr;
  hipStream_t own_coord_ = nullptr;  // the coordinator stream in place of the NULL stream (set_stream)
  bool msg_wt_ = true;  // remote messages written through at system scope (EpochArgs::dst_sys)
  bool pub_local_ = true;  // MPA_PUB_LOCAL=0: every task publishes at system scope
  // a task's reply stays on this GPU for this process's later kernels (SOLO, rank 0's own
  // workers); a worker process's replies go to rank 0 (LsqTask::pub_local)
  int pub_local() const { return pub_local_ && role_ != SERVER ? 1 : 0; }
  unsigned long long* flags_ = nullptr;
  unsigned* err_ = nullptr;
  unsigned* err_dev_ = nullptr;
  unsigned long long* cancel_ = nullptr;  // server: cancel words of armed tasks (host-pinned)
  bool xgmi_ = true;                      // MPA_XGMI=0: payloads always via the host mailbox
  uint32_t* ctr_ = nullptr;
  uint32_t* ticket_ = nullptr;
  uint32_t ticket_count_ = 0;
  // fused tail (maybe_ahead): the next least-squares launch carries tail_args_ (tail_next_);
  // the epoch step of the next ahead epoch is already enqueued in a tail (tail_pending_)
  uint32_t* tail_ctr_ = nullptr;
  bool fused_tail_ = true;  // MPA_TAIL=0: a separate epoch kernel every epoch
  // MPA_LSQP_SHARE=1: a single-pass launch's grid is dealt as if every local batched worker
  // ran in it (off: batches share the coordinator stream, so a partial grid idles CUs; c5
  // 19.9 vs 11.1 ms per epoch, profiles/r02_c5_lsqp_tuning.txt)
  bool lsqp_share_ = false;
  int here_count_ = 0;       // workers this process serves
  // N > 1: on rank 0, tasks of a k-of-n call run on launch streams instead of
  // behind the epoch step on the coordinator's stream (split_local_), so the next step never
  // waits for rank 0's own straggler (MPA_SPLIT_LOCAL=0: as before); and, opt-in
  // (MPA_RESERVE_CUS=1), every task stream on rank 0's GPU -- rank 0's, and a worker process's
  // that shares the GPU (the one-GPU rehearsal) -- leaves CU 0 of each XCD to the coordinator's
  // stream (reserve_cus_), so the step finds a CU while a task holds the rest (lsqp4 fills every
  // CU's register file: its grid shrinks to fit)
  hipEvent_t switch_ev_ = nullptr;  // set_stream: the old coordinator stream's tail
  // N > 1, device payload path: each remote worker's completion word has a device copy after
  // its reply inbox in rank 0's memory (publish_peer), which rank 0's kernels poll instead of
  // the host-memory word (MPA_DONE_DEV=0: the host word only, as before round 6)
  bool done_dev_ = true;
  size_t done_off() const { return region_ ? (region_->max_msg() + 255) / 256 * 256 : 0; }
  // the server's task: rank 0's device done word of worker w (mapped by IPC), or null
  unsigned long long* peer_done(const HipWorker& w) const {
    return role_ == SERVER && done_dev_ && w.path_dev && w.peer_reply
               ? reinterpret_cast<unsigned long long*>(w.peer_reply + done_off())
               : nullptr;
  }
  // rank 0: the word its kernels poll for remote worker w's completion
  const unsigned long long* remote_done_word(const HipWorker& w) const {
    return done_dev_ && w.path_dev && w.reply_inbox
               ? reinterpret_cast<const unsigned long long*>(w.reply_inbox + done_off())
               : region_->dev(&w.box->done);
  }
  bool split_local_ = false;
  bool reserve_cus_ = false;
  bool hold_ok_ = true;     // MPA_HOLD=0: a stale re-dispatch launches at once (flush_stale)
  bool hold_next_ = false;  // set while flush_stale() flushes
  bool may_hold_ = false;   // this call's wait completes without the held tasks (set_wait_hold)
  const void* checked_bufs_[4] = {};  // the buffer pointers check_buffers() last accepted
  std::vector<int64_t> held_;  // held re-dispatches, launched with the next batch
  // held re-dispatches: held, later joined a batched launch, launched on their own
  int64_t n_held_ = 0, n_held_joined_ = 0, n_held_alone_ = 0;
  bool lsqp8_ = false;  // MPA_LSQP=8: the eight-wave single pass (lsqp_kernel.hip)
  bool lsqc_ = false;   // MPA_LSQP=c: the column-pair single pass (lsqc_kernel.hip)
  int lsqc_la_ = 2;     // MPA_LSQC_LA: its phase-1 lookahead in blocks (2; 1 for A/B)
  // lsqp L2 prefetch lead in blocks (MPA_LSQP_PF; 0 = off; unset: 1 for lsqp4, 0 for the
  // eight-wave cut).  lsqp4: 1 block 8.47 ms vs 9.50 without, 2-4 slower (L2 thrash);
  // profiles/r02_c5_lsqp_tuning.txt
  int lsqp_pfd_ = -1;
  bool tail_next_ = false, tail_pending_ = false;
  // fused head (flush): the next least-squares launch runs this epoch's step first
  bool fused_head_ = true;  // MPA_HEAD=0: the step runs as its own epoch kernel
  bool head_next_ = false;
  size_t head_ranks_ = 0;
  EpochArgs head_args_{};
  uint32_t* head_word_ = nullptr;
  uint32_t head_token_ = 0;
  int64_t n_head_ = 0, n_epoch_ = 0;
  bool head_fits(const std::vector<int64_t>& posted, const UpdateSpec& u) const;
  uint32_t next_head_token() {
    head_token_ = (head_token_ + 1) & ~kHeadCancel;
    if (head_token_ == 0) head_token_ = 1;
    return head_token_;
  }
  // Pre-armed launches (the native descent loop at nwait < n, every epoch a fused-head launch
  // of the whole pool: c1): right after an epoch's launch the next one is enqueued behind it,
  // its tasks numbered one ahead, its workgroup 0 waiting on a pinned mailbox; the next flush
  // that posts the same workers writes the epoch step's arguments there and releases it
  // (pre_consume), anything else cancels it first (cancel_pre).  The host's launch call and
  // the command processor's dispatch leave the epoch's critical path (7.9 vs 2.8 us round
  // trip, profiles/r03_launch_cost.txt).  MPA_PREARM=0: off.
  struct PreMailbox {
    unsigned long long go;
    unsigned long long pad[7];
    EpochArgs ep;
  };
  bool prearm_ = true;
  bool prearm_loop_ = false;  // the running descent loop allows it (set_defer_end_flush)
  bool pre_active_ = false;
  bool pre_vec_ = false;
  PreMailbox* pre_mb_ = nullptr;  // host-pinned, coherent
  unsigned long long pre_token_ = 0;
  std::vector<int64_t> pre_ranks_, last_head_ranks_;
  std::vector<uint64_t> pre_seq_;
  std::vector<const uint8_t*> pre_x_;
  std::vector<uint8_t*> pre_out_;
  int64_t n_prearmed_ = 0, n_pre_cancel_ = 0, pre_count_ = 0;
  bool time_next_ = false;  // the next normal launch is timed (pre-arming skipped for it)
  EpochArgs pre_pred_{};    // the step the pre-armed launch carries as its prediction
  bool pre_same_ = true;    // MPA_PRESAME=0: always release through the mailbox
  int64_t n_pre_same_ = 0;
  bool pre_consume();
  void maybe_prearm(int dtype);
  // Held stale re-dispatches in the descent loop (flush_stale): their message copies (and the
  // call's pending harvests) join the next flush's epoch step, before its update (EpochArgs
  // dst0), instead of an exchange launch of their own; run_deferred() issues them as that
  // launch when something else must run first (a held task released, a step that cannot
  // carry them).  {message source, slot, bytes}
  struct Deferred0 {
    const uint8_t* src;
    uint8_t* dst;
    size_t bytes;
  };
  std::vector<Deferred0> stale_deferred_;
  int64_t n_deferred_ = 0;
  bool defer_ok_ = true;  // MPA_DEFER=0: a held re-dispatch's copies go out at once
  bool defer_stale();
  void run_deferred();
  bool deferred_fit(const UpdateSpec& u) const {
    const uint8_t* msg = u.msg_bf16 ? reinterpret_cast<const uint8_t*>(u.mirror) : static_cast<const uint8_t*>(u.x);
    for (const auto& d : stale_deferred_)
      if (d.src != msg || d.bytes != b_.sl) return false;
    return true;
  }
  std::vector<int64_t> launch_ranks() const {  // the ranks launch_local would launch together
    std::vector<int64_t> r(held_);
    r.insert(r.end(), posts_.begin(), posts_.end());
    return r;
  }
  void cancel_pre() {
    if (!pre_active_) return;
    __atomic_store_n(&pre_mb_->go, pre_token_ | kPreCancel, __ATOMIC_RELEASE);
    pre_active_ = false;
    ++n_pre_cancel_;
  }
  size_t tail_ranks_ = 0;  // local tasks of the launch that carries the tail
  EpochArgs tail_args_{};
  // rank 0: the completion words of the epoch's remote workers the tail waits for
  int tail_nwait_ = 0;
  const unsigned long long* tail_word_[kMaxEpochChunks] = {};
  unsigned long long tail_target_[kMaxEpochChunks] = {};
  hipEvent_t xfer_ev_ = nullptr;
  double rt_hz_ = 100e6;
  double timeout_s_ = 600.0;
  std::vector<int64_t> posts_;
  std::vector<Harvest> harv_;
  CallBufs b_;
  std::vector<Harvest> call_posts_;  // (slot, rank) of every post() of the current call
  bool defer_end_ = false;
  bool has_update_ = false;
  size_t harv_before_ = 0;  // harvests staged before the pending update
  UpdateSpec upd_;
  int64_t ahead_left_ = 0;
  UpdateSpec ahead_pred_, ahead_upd_;
  CallBufs ahead_bufs_;
  bool ahead_update_ = false;
  std::atomic<bool> timing_{false};  // read by the straggler timer thread's launches
  int timing_period_ = 1;
  std::atomic<uint64_t> t_seq_{0};  // task launches seen while timing (the timer thread launches too)
  std::atomic<int64_t> n_task_launches_{0};  // every task launch ("task_launches")
  uint64_t x_seq_ = 0;              // epoch kernels seen while timing
  bool sample_task(int64_t armed_rank) {
    if (!timing_) return false;
    return armed_rank != 0 || timing_period_ <= 1 || t_seq_.fetch_add(1) % uint64_t(timing_period_) == 0;
  }
  bool debug_ = false;
  int arm_mode_ = 0;
  int arm_depth_env_ = 0;  // MPA_ARM_DEPTH (0: arm_depth()'s default)
  bool arm_wave_ = true;  // MPA_ARM_WAIT: an armed task waits behind a one-wave door_wait_kernel
  bool arm_force_ = false;  // MPA_ARM_WAIT_FORCE=1 (measurement build): in-kernel waits on rank 0's GPU too
  bool batch_gather_ = true;  // MPA_GATHER=0: a server launches whatever one doorbell scan found
  // undelayed task batches run on the coordinator stream behind the exchange that delivered
  // their messages (MPA_COORD_BATCH=0: on a launch stream behind a cross-queue event wait,
  // which measured 75-200 us per hand-off on the k-of-n path, profiles/r01_c1_timeline.txt)
  bool coord_batches_ = true;
  std::vector<TimedLaunch> timed_;
  std::vector<hipEvent_t> event_pool_;
  int64_t t_launches_ = 0;
  double t_ms_ = 0, t_bytes_ = 0;
  std::vector<std::pair<double, double>> t_iv_;  // launch intervals (ms from anchor_)
  hipEvent_t anchor_ = nullptr;
  std::vector<hipStream_t> launch_streams_;
  size_t next_launch_ = 0;
  std::mutex tm_mu_;  // timed_ / event_pool_ (the timer thread also launches)
  // straggler timer thread
  std::thread timer_;
  std::mutex tmu_;
  std::condition_variable tcv_, tidle_;
  std::vector<Deferred> deferred_;
  bool tstop_ = false, tbusy_ = false;
  // the heap front's due time (~0: none) and a stop request, readable without tmu_: the timer's
  // final spin watches them, so an earlier deadline deferred during the spin, or stop_timer,
  // ends the spin at once
  std::atomic<uint64_t> tfront_{~0ull};
  std::atomic<bool> tstop_spin_{false};
  std::atomic<bool> tfailed_{false};
  std::mutex tfail_mu_;
  std::string tfail_msg_;
  std::atomic<int64_t> n_timer_late_{0};  // deferred launches issued > 1 ms after due (counter 'timer_late')
  // Injected delays (launch_tasks): MPA_DELAY=timer the host timer always, =device a device
  // deadline wherever the worker's stream is its own, unset (auto) a device deadline where no
  // caller work on the legacy NULL stream can meet it (a CU-masked worker stream is a blocking
  // stream: every NULL-stream command would wait for the sleeping straggler, round 4's
  // objection): in a worker process, inside the native descent loop, or for a caller on a stream
  // of its own; the host timer otherwise
  int delay_mode_ = 0;                     // 0 auto, 1 timer, 2 device
  bool caller_null_ = true;                // the caller's stream (set_stream) is the NULL stream
  int64_t delay_lead_ns_ = kDelayLeadNs;   // MPA_DELAY_LEAD_NS: the timer's launch overhead, out of its sleep
  int64_t deadline_lead_ns_ = kDeadlineLeadNs;
  // host <-> device clock map (steady-clock ns, s_memrealtime ticks): the first sample and the
  // latest (ck_mu_: the sampling thread writes them)
  int64_t ck_t0_ = 0, ck_n0_ = 0, ck_t1_ = 0, ck_n1_ = 0;
  std::atomic<int64_t> n_clock_samples_{0};
  std::mutex ck_mu_;
  std::mutex tmu_ck_;  // the sampling thread's sleep / stop
  std::thread ck_thread_;
  std::condition_variable ck_cv_;
  bool ck_stop_ = false;
  hipStream_t ck_stream_ = nullptr;
  uint64_t* ck_probe_ = nullptr;  // host-pinned word the clock probes store into
  bool device_delay_ok(hipStream_t s) const;
  unsigned long long device_deadline(int64_t host_ns);
  // one probe round trip on `s` (idle): (device ticks, host ns) at its midpoint, returns the round
  // trip in ns (or -1: the probe had not landed after 100 ms)
  int64_t clock_sample(hipStream_t s, int64_t* ticks, int64_t* ns);
  void clock_loop();
  void stop_clock();
  int64_t n_sleeps_ = 0;  // delayed tasks queued behind a device deadline
  int64_t n_armed_ = 0;   // server: tasks launched device-armed (counter 'armed')  // delayed tasks (a sleep kernel before the task, counter 'sleeps')

 public:
  void init_ticket() {
    ticket_ = ctr_ + kLsqCtrPerTask * nworkers_;
    tail_ctr_ = ticket_ + 1;
    head_word_ = ticket_ + 2;
  }
};

}  // namespace mpa
