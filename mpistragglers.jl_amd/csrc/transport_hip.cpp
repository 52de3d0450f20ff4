// HIP transport: the MPI point-to-point layer of MPIAsyncPools.jl replaced by device work.
//
//   MPI.Isend(isendbufs[i]) + MPI.Irecv!(irecvbufs[i])   (src/MPIAsyncPools.jl:137-138)
//     -> post(): deferred to flush(), where ONE exchange kernel on the coordinator stream
//        copies sendbuf into every posted slot of isendbuf (and into the mailbox of every
//        worker served by another process, whose doorbell the same kernel rings once its
//        copies are released), performs the pending harvest copies, and one event orders
//        the task launches of the workers served here after it.
//   MPI.Test! / MPI.Waitany! / MPI.Waitall!               (:99, :161, :212)
//     -> loads of the worker's host-visible completion word, which the task kernel's last
//        workgroup publishes with a system-scope release (no hipEventQuery, no sync call).
//   recvbufs[i] .= irecvbufs[i]                          (:108, :167, :216)
//     -> deferred and batched into the next exchange kernel on the coordinator stream,
//        which is ordered before any later re-post to that worker (the reference's
//        program order, :167 before :182-183).
//
// Roles.  SOLO: one process, every worker on this GPU.  COORD: rank 0 of a multi-process
// communicator (one process per GPU); workers placed on rank 0 run
// here, the others are reached through shared-memory mailboxes (shm.hpp).  SERVER: a
// worker process; serve() watches the doorbells of its workers and launches their tasks,
// whose replies and completion words land in the mailboxes.
//
// Streams.  Every worker stream and launch stream is CU-masked with every CU enabled:
// such a stream gets an HSA queue of its own, whereas plain streams beyond
// GPU_MAX_HW_QUEUES share queues and HIP serialises kernels of a shared queue
// (profiles/r01_hw_queues.txt), which would let one straggler hold back another worker.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
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

int g_lsq_grid = 0;  // mpa_tune("lsq_grid", G): workgroups per least-squares launch (0 = default)
// A/B switches of the measurement build only (make MEASURE=1): the product reads none of
// them, so the shipped behaviour cannot be switched off by an environment variable
const char* measure_env(const char* name) { return MPA_MEASURE ? std::getenv(name) : nullptr; }
// rank 0 waits for remote completions of a launched-ahead epoch with one wait_words_kernel
// (default) or, MPA_WAIT_VALUE_OPS=1, one hipStreamWaitValue64 per remote worker (round 1)
const bool g_wait_value_ops = [] { const char* e = measure_env("MPA_WAIT_VALUE_OPS"); return e && *e == '1'; }();

namespace {

using Clock = std::chrono::steady_clock;
// workgroups per least-squares launch: 192 (24 per XCD, 3/4 of the CUs) streams the c2
// batch at 7.1-7.2 TB/s against 6.7-6.8 at 512 and 7.0 at 256 (profiles/r01_tune_sweep4_grid.jsonl,
// same-box bench A/B in profiles/r01_lsq_grid_ab.txt: c2 +6-7 %, c3/c4 unchanged); the read
// probe (mpa_read_bandwidth) shows the same shape: fewer, longer streams read faster
constexpr int kDefaultLaunchGrid = 192;
constexpr int kWideResidGrid = 1024;  // wide rows: pass-1 workgroups per launch (a wave per row)
constexpr int kSlabGridCap = kLsqMaxGrid;  // most workgroups a single task may be given
constexpr int kLaunchStreams = 2;
// batched multi-iterate task: pass-1 / pass-2 workgroups per launch (= resident: 1 x 512 /
// 2 x 256 threads per CU by VGPRs), and the most row ranges a pass-2 task is split into
constexpr int kLsqbGrid1 = 512;  // two 8-wave workgroups per CU: pass 1 4.74-4.88 -> 5.11 TB/s (profiles/r01_lsqb_grid.txt)
constexpr int kLsqbGrid2 = 512;
constexpr int kLsqbRangeCap = 128;
constexpr int kLsqfGrid = 256;  // single-pass batched launch: one 768-thread workgroup per CU
constexpr size_t kLsqfCtrBytes = 64 + 16 * sizeof(unsigned long long);

bool env_off(const char* name) {
  const char* e = std::getenv(name);
  return e && *e == '0';
}

// c5 launch grids (MPA_LSQB_GRID1 / MPA_LSQB_GRID2 override them for measurement)
int lsqb_grid(int pass) {
  static const int g1 = [] { const char* e = measure_env("MPA_LSQB_GRID1"); return e ? std::max(8, std::atoi(e)) : kLsqbGrid1; }();
  static const int g2 = [] { const char* e = measure_env("MPA_LSQB_GRID2"); return e ? std::max(8, std::atoi(e)) : kLsqbGrid2; }();
  return pass == 1 ? g1 : g2;
}

// Process-wide pool of CU-masked streams: communicators come and go (tests create many),
// but the HSA queues behind their streams are a bounded hardware resource, so a destroyed
// comm returns its streams here and the next comm reuses them instead of growing the
// process's queue count (more queues than the hardware maps at once are time-sliced).
std::mutex g_stream_mu;
std::vector<std::pair<int, hipStream_t>> g_free_streams;

// The pooled streams (and their HSA queues) are destroyed at process exit, before the HIP
// runtime's own teardown (atexit handlers run in reverse registration order, and the runtime
// registers its teardown when it is loaded, before the first stream here): a profiler that
// tears down while queues are still alive crashed in __cxa_finalize.
void destroy_pooled_streams() {
  std::lock_guard<std::mutex> lk(g_stream_mu);
  for (auto& ds : g_free_streams) (void)hipStreamDestroy(ds.second);
  g_free_streams.clear();
}

hipStream_t make_queue_stream(int device) {
  static const bool registered = (std::atexit(destroy_pooled_streams), true);
  (void)registered;
  {
    std::lock_guard<std::mutex> lk(g_stream_mu);
    for (size_t k = 0; k < g_free_streams.size(); ++k)
      if (g_free_streams[k].first == device) {
        hipStream_t s = g_free_streams[k].second;
        g_free_streams.erase(g_free_streams.begin() + std::ptrdiff_t(k));
        return s;
      }
  }
  hipDeviceProp_t p;
  HIPCHECK(hipGetDeviceProperties(&p, device));
  const int cus = p.multiProcessorCount;
  std::vector<uint32_t> mask(size_t((cus + 31) / 32), 0xFFFFFFFFu);
  if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
  hipStream_t s = nullptr;
  HIPCHECK(hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()));
  return s;
}

void release_queue_stream(int device, hipStream_t s) {
  (void)hipStreamSynchronize(s);
  std::lock_guard<std::mutex> lk(g_stream_mu);
  g_free_streams.push_back({device, s});
}

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
  // server, pre-armed task (serve()): armed = task `seq` is queued behind its doorbell;
  // cancel word (host-pinned, device view) of the armed task; counter bases to restore
  // if cancelled
  bool armed = false;
  unsigned long long* cancel_host = nullptr;
  unsigned long long* cancel_dev = nullptr;
  // coordinator, launch-ahead: the next post / harvest of this worker is already enqueued
  bool preposted = false, preharvest = false;
  uint32_t arm_sbase = 0, arm_tbase = 0, arm_fsbase = 0, arm_ftbase = 0;
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

class HipComm final : public Comm {
 public:
  enum Role { SOLO, COORD, SERVER };

  HipComm(int64_t n, const int* devices, const int* placement, int my_rank, ShmRegion* region)
      : Comm(n), w_(size_t(n)), region_(region), my_rank_(my_rank) {
    role_ = !region ? SOLO : my_rank == 0 ? COORD : SERVER;
    HIPCHECK(hipGetDevice(&dev_));
    for (int64_t i = 0; i < n; ++i) {
      HipWorker& w = w_[size_t(i)];
      const int host_rank = placement ? placement[i] : 0;
      w.here = host_rank == my_rank_;
      w.remote = role_ == COORD && !w.here;
      if (devices && w.here && devices[i] != dev_)
        fail(MPA_ARGUMENT_ERROR, "worker %lld on device %d: a process serves the workers of its own device (%d); "
             "workers of other devices are served by their own processes (DESIGN.md §Multi-GPU)",
             (long long)(i + 1), devices[i], dev_);
    }
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&flags_), sizeof(unsigned long long) * size_t(n + 1),
                           hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(flags_, 0, sizeof(unsigned long long) * size_t(n + 1));
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&err_), 64, hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(err_, 0, 64);
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&cancel_), sizeof(unsigned long long) * size_t(n + 1),
                           hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(cancel_, 0, sizeof(unsigned long long) * size_t(n + 1));
    xgmi_ = !env_off("MPA_XGMI");
    // per-task tree counters, then the doorbell ticket and the fused-tail counter
    HIPCHECK(hipMalloc(&ctr_, sizeof(uint32_t) * (kLsqCtrPerTask * size_t(n) + 2)));
    HIPCHECK(hipMemset(ctr_, 0, sizeof(uint32_t) * (kLsqCtrPerTask * size_t(n) + 2)));
    err_dev_ = err_;
    if (region_) {
      if (region_->nworkers() != n) fail(MPA_ARGUMENT_ERROR, "shared memory holds %lld workers, comm has %lld",
                                         (long long)region_->nworkers(), (long long)n);
      if (role_ == SERVER) err_dev_ = region_->dev(&region_->header()->err);
    }
    for (int64_t r = 1; r <= n; ++r) {
      HipWorker& w = w_[size_t(r - 1)];
      if (region_ && (w.remote || (role_ == SERVER && w.here))) {
        w.box = region_->box(r);
        w.box_msg_dev = region_->dev(region_->msg(r));
        w.box_reply_dev = region_->dev(region_->reply(r));
        w.box_door_dev = region_->dev(&w.box->doorbell);
      }
      if (role_ == SERVER && w.here) {
        w.flag_host = &w.box->done;
        w.flag_dev = region_->dev(&w.box->done);
        w.box->server_dev = dev_;
        w.xslot = static_cast<uint8_t*>(ipc_alloc(region_->max_msg(), w.box->msg_handle, &w.box->msg_ipc));
        w.cancel_host = &cancel_[r - 1];
        w.cancel_dev = &cancel_[r - 1];
      } else if (w.remote) {
        w.flag_host = &w.box->done;
        w.box->coord_dev = dev_;
        w.reply_inbox = static_cast<uint8_t*>(ipc_alloc(region_->max_msg(), w.box->reply_handle, &w.box->reply_ipc));
      } else {
        w.flag_host = &flags_[r - 1];
        w.flag_dev = &flags_[r - 1];
      }
    }
    // Streams are HSA queues of their own, and creating one takes milliseconds, so none is
    // created inside a timed schedule: a worker's stream when its task is registered
    // (on_task_changed), the launch streams here where they can be used (a worker process
    // serving several workers batches staged tasks on them).  A process serving ONE
    // pre-armed worker (N = 8) then holds one queue, not four, which matters when the
    // GPU's hardware queue slots are shared; MPA_EAGER_STREAMS=1 creates every stream up
    // front (the round-1 behaviour, for A/B measurements).
    int here_count = 0;
    for (const auto& w : w_) here_count += w.here;
    const char* eager = measure_env("MPA_EAGER_STREAMS");
    if (eager && *eager == '1') {
      for (auto& w : w_)
        if (w.here) worker_stream(w);
      launch_stream(kLaunchStreams - 1);
    } else if (role_ == SERVER && here_count > 1) {
      launch_stream(kLaunchStreams - 1);
    }
    HIPCHECK(hipEventCreateWithFlags(&xfer_ev_, hipEventDisableTiming));
    int khz = 0;
    HIPCHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_));
    rt_hz_ = khz > 0 ? double(khz) * 1e3 : 100e6;
    const char* t = std::getenv("MPA_WAIT_TIMEOUT_S");
    timeout_s_ = t ? std::atof(t) : 600.0;
    // unset / 0: never pre-arm; 1: arm every eligible worker; 2: when a process serves one
    const char* arm = std::getenv("MPA_ARM");
    arm_mode_ = arm && *arm == '1' ? 1 : arm && *arm == '2' ? 2 : 0;
    const char* cb = measure_env("MPA_COORD_BATCH");
    coord_batches_ = !(cb && *cb == '0');
    fused_tail_ = !env_off("MPA_TAIL");
    { const char* e = measure_env("MPA_LSQP_SHARE"); lsqp_share_ = e && *e == '1'; }
    {
      const char* e = measure_env("MPA_LSQP");  // the product's MPA_LSQP=0 is read where it applies
      lsqp8_ = e && *e == '8';
      lsqc_ = e && *e == 'c';
      const char* la = measure_env("MPA_LSQC_LA");
      lsqc_la_ = la && *la == '1' ? 1 : 2;
    }
    hold_ok_ = !env_off("MPA_HOLD");
    { const char* e = measure_env("MPA_GATHER"); batch_gather_ = !(e && *e == '0'); }
    if (const char* e = measure_env("MPA_LSQP_PF")) lsqp_pfd_ = std::max(0, std::min(8, std::atoi(e)));
    const char* dbg = std::getenv("MPA_DEBUG");
    debug_ = dbg && *dbg == '1';
    if (debug_ && region_) {
      std::fprintf(stderr, "[mpa role %d rank %d] shm header %p (device %p)\n", int(role_), my_rank_,
                   (void*)region_->header(), (void*)region_->dev(region_->header()));
      describe("shm", region_->dev(region_->header()));
    }
    HIPCHECK(hipDeviceSynchronize());
  }

  ~HipComm() override {
    try {
      release_held();
      disarm_all();
    } catch (...) {
    }
    stop_timer();
    (void)hipDeviceSynchronize();
#if MPA_MEASURE
    if (const char* d = measure_env("MPA_LSQF_DBG"); d && (std::atoi(d) & 16)) lsqf_prof_dump();
#endif
    for (auto& w : w_) {
      if (w.slab) (void)hipFree(w.slab);
      if (w.wctr) (void)hipFree(w.wctr);
      if (w.lsqb_R) (void)hipFree(w.lsqb_R);
      if (w.lsqb_slab) (void)hipFree(w.lsqb_slab);
      if (w.lsqb_ctr) (void)hipFree(w.lsqb_ctr);
      if (w.lsqf_x) (void)hipFree(w.lsqf_x);
      if (w.lsqf_flag) (void)hipFree(w.lsqf_flag);
      if (w.lsqf_ctr) (void)hipFree(w.lsqf_ctr);
      if (w.lsqq_ctr) (void)hipFree(w.lsqq_ctr);
      if (w.lsqp_slab) (void)hipFree(w.lsqp_slab);
      if (w.lsqp_ctr) (void)hipFree(w.lsqp_ctr);
      if (w.lsqc_xg) (void)hipFree(w.lsqc_xg);
      if (w.peer_msg) (void)hipIpcCloseMemHandle(w.peer_msg);
      if (w.peer_reply) (void)hipIpcCloseMemHandle(w.peer_reply);
      if (w.xslot) (void)hipFree(w.xslot);
      if (w.reply_inbox) (void)hipFree(w.reply_inbox);
      if (w.stream) release_queue_stream(dev_, w.stream);
    }
    for (auto& s : launch_streams_) release_queue_stream(dev_, s);
    for (auto& t : timed_) {
      (void)hipEventDestroy(t.start);
      (void)hipEventDestroy(t.stop);
    }
    for (auto e : event_pool_) (void)hipEventDestroy(e);
    if (ctr_) (void)hipFree(ctr_);
    if (flags_) (void)hipHostFree(flags_);
    if (err_) (void)hipHostFree(err_);
    if (cancel_) (void)hipHostFree(cancel_);
    if (xfer_ev_) (void)hipEventDestroy(xfer_ev_);
    delete region_;
  }

  int transport() const override { return MPA_TRANSPORT_HIP; }
  void set_stream(hipStream_t s) { coord_ = s; }
  hipStream_t stream() const { return coord_; }

  void begin_call(const CallBufs& b) override {
    if (role_ == SERVER) fail(MPA_ERROR, "asyncmap!/waitall! run on rank 0; this process serves workers (mpa_comm_serve)");
    b_ = b;
    call_posts_.clear();
  }

  void post(int64_t i, int64_t rank, int64_t tag) override {
    (void)tag;
    if (shutdown_) fail(MPA_ERROR, "comm has been shut down");
    HipWorker& w = w_[size_t(rank - 1)];
    call_posts_.push_back({i, rank});
    if (w.preposted) {
      // enqueued one epoch ahead (enqueue_ahead): same slot and buffers, nothing to launch
      if (w.slot != i || w.sl != b_.sl || w.rl != b_.rl || b_.isendbuf != ahead_bufs_.isendbuf ||
          b_.irecvbuf != ahead_bufs_.irecvbuf || b_.recvbuf != ahead_bufs_.recvbuf || b_.sendbuf != ahead_bufs_.sendbuf)
        fail(MPA_ERROR, "launch-ahead: the call posts worker %lld differently from the epoch enqueued ahead",
             (long long)rank);
      w.preposted = false;
      w.seq += 1;
      return;
    }
    if (w.remote) {
      if (!w.path_known) decide_path(rank);
      if (b_.sl > region_->max_msg() || b_.rl > region_->max_msg())
        fail(MPA_DIMENSION_MISMATCH, "messages of %zu / %zu bytes exceed the communicator's mailbox of %zu bytes",
             b_.sl, b_.rl, region_->max_msg());
      w.box->msg_bytes = b_.sl;
      w.box->reply_bytes = b_.rl;
    } else {
      check_task(rank, tasks_[size_t(rank - 1)], b_.sl, b_.rl);
      w.x = b_.isendbuf + size_t(i) * b_.sl;
      w.out = b_.irecvbuf + size_t(i) * b_.rl;
    }
    w.slot = i;
    w.sl = b_.sl;
    w.rl = b_.rl;
    w.seq += 1;
    posts_.push_back(rank);
  }

  void harvest(int64_t i, int64_t rank) override {
    HipWorker& w = w_[size_t(rank - 1)];
    if (w.preharvest) {  // already in the epoch kernel enqueued ahead
      w.preharvest = false;
      return;
    }
    harv_.push_back({i, rank});
  }

  bool test(int64_t i, int64_t rank) override {
    (void)i;
    return done(rank);
  }

  int64_t waitany(int64_t n, const int64_t* ranks, const uint8_t* live) override {
    bool any = false;
    for (int64_t i = 0; i < n; ++i) any |= live[i] != 0;
    if (!any) return -1;
    if (!held_.empty() && !may_hold_) {  // the wait would block: held launches go first
      for (int64_t i = 0; i < n; ++i)
        if (live[i] && done(ranks[i])) return i;
      release_held();
    }
    const auto t0 = Clock::now();
    for (uint64_t spins = 0;; ++spins) {
      for (int64_t i = 0; i < n; ++i)
        if (live[i] && done(ranks[i])) return i;
      if ((spins & 0xFFF) == 0xFFF) watchdog(t0);
      __builtin_ia32_pause();
    }
  }

  void waitall(int64_t n, const int64_t* ranks, const uint8_t* live) override {
    release_held();
    const auto t0 = Clock::now();
    for (int64_t i = 0; i < n; ++i) {
      if (!live[i]) continue;
      for (uint64_t spins = 0; !done(ranks[i]); ++spins) {
        if ((spins & 0xFFF) == 0xFFF) watchdog(t0);
        __builtin_ia32_pause();
      }
    }
  }

  void flush() override {
    if (posts_.empty() && harv_.empty() && !has_update_) {
      maybe_ahead();
      return;
    }
    if (timing_) reap_timing(false);
    if (has_update_ && fused_ok(upd_, posts_)) {
      emit_epoch(harv_, harv_before_, posts_, upd_, coord_);
    } else {
      ExchangeBuilder xb(ticket_, &ticket_count_, coord_);
      size_t h0 = 0;
      if (has_update_) {  // unfused: harvests before the update, the update, then the rest
        for (; h0 < harv_before_; ++h0) add_harvest(xb, harv_[h0]);
        xb.launch();
        launch_update(upd_);
      }
      for (size_t k = h0; k < harv_.size(); ++k) add_harvest(xb, harv_[k]);
      for (int64_t rank : posts_) {
        const HipWorker& w = w_[size_t(rank - 1)];
        uint8_t* slot = b_.isendbuf + size_t(w.slot) * b_.sl;
        if (w.remote) {
          xb.reserve(2, 1);
          xb.copy(b_.sendbuf, slot, b_.sl);
          xb.copy(b_.sendbuf, msg_dst(w), b_.sl);
          xb.door(w.box_door_dev, w.seq);
        } else {
          xb.copy(b_.sendbuf, slot, b_.sl);
        }
      }
      xb.launch();
    }
    has_update_ = false;
    harv_.clear();
    launch_local(posts_);
    posts_.clear();
    maybe_ahead();
  }

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
  void flush_stale() override {
    hold_next_ = hold_ok_;
    flush();
    hold_next_ = false;
  }
  void set_wait_hold(bool may_hold) override { may_hold_ = may_hold; }
  void release_held() {
    if (held_.empty()) return;
    std::vector<int64_t> h;
    h.swap(held_);
    n_held_alone_ += int64_t(h.size());
    launch_tasks(h, /*staged=*/false);
  }

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
  void set_defer_end_flush(bool on) {
    defer_end_ = on;
    if (!on) tail_next_ = tail_pending_ = false;  // the descent loop ended (or failed)
  }
  void stage_update(const UpdateSpec& u) {
    if (ahead_update_) {  // enqueued ahead with the predicted weights: they must match
      ahead_update_ = false;
      if (u.w != ahead_upd_.w || u.x != ahead_upd_.x || u.eta != ahead_upd_.eta || u.elems != ahead_upd_.elems)
        fail(MPA_ERROR, "launch-ahead: the iterate update differs from the one enqueued ahead");
      return;
    }
    if (has_update_) flush();
    upd_ = u;
    has_update_ = true;
    harv_before_ = harv_.size();
  }
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

  void shutdown() override {
    gate_off();
    release_held();
    if (role_ != SERVER) {
      const auto t0 = Clock::now();
      for (int64_t r = 1; r <= nworkers_; ++r) {
        if (!w_[size_t(r - 1)].here && !w_[size_t(r - 1)].remote) continue;
        for (uint64_t spins = 0; !done(r); ++spins) {
          if ((spins & 0xFFF) == 0xFFF) watchdog(t0);
          __builtin_ia32_pause();
        }
      }
      if (region_) __atomic_store_n(&region_->header()->shutdown, 1ull, __ATOMIC_RELEASE);
    }
    drain_deferred();
    for (auto& w : w_)
      if (w.stream) HIPCHECK(hipStreamSynchronize(w.stream));
    for (auto& s : launch_streams_) HIPCHECK(hipStreamSynchronize(s));
    shutdown_ = true;
  }

  void on_task_changed(int64_t rank) override {
    HipWorker& w = w_[size_t(rank - 1)];
    if (!w.here)
      fail(MPA_ARGUMENT_ERROR, "worker %lld is served by another process; register its task there", (long long)rank);
    if (w.seq != uint64_t(tasks_done(rank)))
      fail(MPA_ERROR, "cannot change the task of worker %lld while it has an outstanding request", (long long)rank);
    worker_stream(w);  // outside any timed schedule (delayed and pre-armed tasks run on it)
    const TaskSpec& ts = tasks_[size_t(rank - 1)];
    if (ts.kind == MPA_TASK_LSQ) prepare_lsq(rank, ts);
    if (ts.kind == MPA_TASK_LSQ_BATCH) prepare_lsqb(rank, ts);
  }

  // ---- worker process: watch the doorbells of the workers served here ----
  // Least-squares workers without a delay schedule are PRE-ARMED: their next task is
  // already queued on the worker's own stream behind hipStreamWaitValue64 on the mailbox
  // doorbell, so the GPU starts it when rank 0's exchange kernel rings (3.2 us ring -> task
  // start, against 13.4 us for host polling + launch; profiles/r01_probe_waitvalue.txt).
  // Other workers (the reference's test programs, injected delays) are launched by this
  // thread when it sees their doorbell.  serve() returns at pause / shutdown after
  // disarming: the pending waits are released with kCancelBit and their tasks return
  // without computing or publishing.
  void serve() {
    if (role_ != SERVER) fail(MPA_ERROR, "mpa_comm_serve is for worker processes (rank != 0)");
    ShmHeader* h = region_->header();
    const uint64_t gen0 = __atomic_load_n(&h->gen, __ATOMIC_ACQUIRE);
    const auto t0 = Clock::now();
    struct Disarm {
      HipComm* c;
      ~Disarm() { c->disarm_all(); }
    } disarm_guard{this};
    std::vector<int64_t> fresh;
    for (int64_t r = 1; r <= nworkers_; ++r)
      if (w_[size_t(r - 1)].here && server_path(r) && armable(r)) arm(r);
    for (uint64_t spins = 0;; ++spins) {
      if (__atomic_load_n(&h->shutdown, __ATOMIC_ACQUIRE) || __atomic_load_n(&h->gen, __ATOMIC_ACQUIRE) != gen0) break;
      fresh.clear();
      bool progress = false;
      for (int64_t r = 1; r <= nworkers_; ++r) {
        HipWorker& w = w_[size_t(r - 1)];
        if (!w.here) continue;
        if (!w.path_known) {
          if (server_path(r)) {
            progress = true;
            if (armable(r)) arm(r);
          }
          continue;
        }
        if (w.armed) {
          if (__atomic_load_n(w.flag_host, __ATOMIC_ACQUIRE) < w.seq) continue;
          // the armed task ran: check what rank 0 posted against what it was armed for
          w.armed = false;
          check_task(r, tasks_[size_t(r - 1)], size_t(w.box->msg_bytes), size_t(w.box->reply_bytes));
          progress = true;
          if (armable(r)) arm(r);
          continue;
        }
        const unsigned long long db = __atomic_load_n(&w.box->doorbell, __ATOMIC_ACQUIRE);
        if (db == w.seq) continue;
        if (db != w.seq + 1) fail(MPA_ERROR, "mailbox protocol: worker %lld doorbell %llu after %llu", (long long)r, db, w.seq);
        if (__atomic_load_n(w.flag_host, __ATOMIC_ACQUIRE) != w.seq)
          fail(MPA_ERROR, "mailbox protocol: worker %lld posted while busy", (long long)r);
        w.seq = db;
        w.sl = size_t(w.box->msg_bytes);
        w.rl = size_t(w.box->reply_bytes);
        check_task(r, tasks_[size_t(r - 1)], w.sl, w.rl);
        w.x = w.xslot;
        w.out = reply_dst(w);
        fresh.push_back(r);
      }
      if (!fresh.empty()) {
        // rank 0's exchange kernel rings a flush's doorbells one after another: a scan that
        // caught the first ones looks again for ~2 us before launching, so the flush's tasks
        // here go out as one batch (the c2 N = 2 trace showed them split over two launches)
        if (batch_gather_) {
          const auto g0 = Clock::now();
          while (std::chrono::duration<double, std::micro>(Clock::now() - g0).count() < 2.0) {
            for (int64_t r = 1; r <= nworkers_; ++r) {
              HipWorker& w = w_[size_t(r - 1)];
              if (!w.here || !w.path_known || w.armed || std::find(fresh.begin(), fresh.end(), r) != fresh.end()) continue;
              const unsigned long long db = __atomic_load_n(&w.box->doorbell, __ATOMIC_ACQUIRE);
              if (db != w.seq + 1 || __atomic_load_n(w.flag_host, __ATOMIC_ACQUIRE) != w.seq) continue;
              w.seq = db;
              w.sl = size_t(w.box->msg_bytes);
              w.rl = size_t(w.box->reply_bytes);
              check_task(r, tasks_[size_t(r - 1)], w.sl, w.rl);
              w.x = w.xslot;
              w.out = reply_dst(w);
              fresh.push_back(r);
            }
            int postable = 0;  // workers here that could still be posted (not busy, not armed)
            for (int64_t r = 1; r <= nworkers_; ++r) {
              const HipWorker& w = w_[size_t(r - 1)];
              postable += w.here && w.path_known && !w.armed &&
                          (std::find(fresh.begin(), fresh.end(), r) != fresh.end() ||
                           __atomic_load_n(w.flag_host, __ATOMIC_ACQUIRE) == w.seq);
            }
            if (int(fresh.size()) >= postable) break;  // every worker that could be posted is
            __builtin_ia32_pause();
          }
          std::sort(fresh.begin(), fresh.end());
        }
        if (timing_) reap_timing(false);
        launch_tasks(fresh, /*staged=*/true);
      } else if (!progress) {
        if ((spins & 0xFFF) == 0xFFF) watchdog(t0, /*timeout=*/false);
        __builtin_ia32_pause();
      }
    }
  }

  // ---- pre-armed tasks (server) ----
  // Off by default (MPA_ARM=2: where a process serves ONE worker; MPA_ARM=1: every eligible
  // worker).  The armed launch saves the host's doorbell poll + launch (3.2 vs 13.4 us ring ->
  // start) but its task ran 7-15x longer than the same task launched by the host: every
  // workgroup reads the host-memory go word before it starts (one-GPU N = 2 rehearsal, c1:
  // 134 us with every lane reading, 73 us with one lane per wave, 9.6 us host-launched;
  // 106 vs 48 us per epoch; c2 with 4 armed workers 1.20 vs 0.74 ms; profiles/r02_arm_go_word.txt).
  // With several workers the host-launched path also batches them into one launch
  // (profiles/r01_n2_arm_ab.txt).
  bool armable(int64_t rank) const {
    const TaskSpec& ts = tasks_[size_t(rank - 1)];
    if (arm_mode_ == 0 || !((ts.kind == MPA_TASK_LSQ || ts.kind == MPA_TASK_LSQ_BATCH) && ts.delays_ns.empty()))
      return false;
    if (arm_mode_ == 1) return true;
    int here = 0;
    for (const auto& w : w_) here += w.here;
    return here == 1;
  }
  // local workers that serve() pre-arms: each armed launch gets its share of the launch grid
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

  // queue task seq+1 of `rank` on its stream: wait for the doorbell, stage the message and
  // the doorbell value (the task's go word), run the task
  void arm(int64_t rank) {
    HipWorker& w = w_[size_t(rank - 1)];
    const TaskSpec& ts = tasks_[size_t(rank - 1)];
    const unsigned long long s = w.seq + 1;
    w.arm_sbase = w.lsqb_sbase;
    w.arm_tbase = w.lsqb_tbase;
    w.arm_fsbase = w.lsqf_sbase;
    w.arm_ftbase = w.lsqf_tbase;
    HIPCHECK(hipStreamWaitValue64(worker_stream(w), w.box_door_dev, s, hipStreamWaitValueGte, ~0ull));
    w.seq = s;
    w.sl = task_msg_bytes(ts);
    w.rl = w.sl * (ts.kind == MPA_TASK_LSQ_BATCH ? 2 : 1);
    w.x = w.xslot;
    w.out = reply_dst(w);
    if (!w.path_dev) {  // host mailbox: stage the message into the device slot first
      ExchangeBuilder xb(ticket_, &ticket_count_, w.stream);
      xb.copy(w.box_msg_dev, w.xslot, w.sl);
      xb.launch();
    }
    double bytes = 0;
    if (ts.kind == MPA_TASK_LSQ) {
      LsqBatch b = build_lsq_batch({rank}, ts.dtype, &bytes, armed_share());
      b.t[0].go = w.cancel_dev;
      enqueue_lsq(b, ts.dtype, int(ts.cols), w.stream, bytes, rank);
    } else {
      LsqbLaunch b = build_lsqb_batch({rank}, &bytes, armed_share());
      b.set_go(w.cancel_dev);
      enqueue_lsqb(b, w.stream, bytes, rank);
    }
    w.armed = true;
  }

  // release every pending armed wait: a task whose doorbell rank 0 has not rung is
  // cancelled (cancel word := its seq, then doorbell := seq | kCancelBit to release the
  // wait; both restored once the stream has drained), one already rung completes.  A task
  // cancelled in a race with rank 0's ring did not run: its doorbell is served by the next
  // serve() session (seq rolled back).
  void disarm_all() {
    if (role_ != SERVER) return;
    for (int64_t r = 1; r <= nworkers_; ++r) {
      HipWorker& w = w_[size_t(r - 1)];
      if (!w.here || !w.armed) continue;
      unsigned long long expect = w.seq - 1;
      bool cancelled = false;
      if (__atomic_load_n(&w.box->doorbell, __ATOMIC_ACQUIRE) < w.seq) {
        __atomic_store_n(w.cancel_host, w.seq, __ATOMIC_SEQ_CST);
        cancelled = __atomic_compare_exchange_n(&w.box->doorbell, &expect, w.seq | kCancelBit, false, __ATOMIC_SEQ_CST,
                                                __ATOMIC_SEQ_CST);
      }
      (void)hipStreamSynchronize(w.stream);
      if (cancelled) {
        unsigned long long c2 = w.seq | kCancelBit;  // restore unless rank 0 rang meanwhile
        __atomic_compare_exchange_n(&w.box->doorbell, &c2, w.seq - 1, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
      }
      __atomic_store_n(w.cancel_host, 0ull, __ATOMIC_SEQ_CST);
      if (__atomic_load_n(w.flag_host, __ATOMIC_ACQUIRE) < w.seq) {  // it did not run
        w.seq -= 1;
        w.lsqb_sbase = w.arm_sbase;
        w.lsqb_tbase = w.arm_tbase;
        w.lsqf_sbase = w.arm_fsbase;
        w.lsqf_tbase = w.arm_ftbase;
        void_timing(r);
      }
      w.armed = false;
    }
  }

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
  void launch_local(const std::vector<int64_t>& posted) {
    std::vector<int64_t> here;
    for (int64_t rank : posted) {
      if (w_[size_t(rank - 1)].remote) continue;
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      if (hold_next_ && (ts.kind == MPA_TASK_LSQ || ts.kind == MPA_TASK_LSQ_BATCH) && ts.delays_ns.empty())
      {
        held_.push_back(rank);  // flush_stale(): joins the next batch
        ++n_held_;
      }
      else
        here.push_back(rank);
    }
    if (!here.empty() && !held_.empty() && !hold_next_) {  // held re-dispatches join this batch
      n_held_joined_ += int64_t(held_.size());
      here.insert(here.begin(), held_.begin(), held_.end());
      held_.clear();
    }
    // every task of this call is awaited before the caller enqueues anything else on the
    // coordinator stream: run the batch right behind the exchange on that stream (a
    // cross-queue event wait costs ~35 us per epoch, profiles/r01_c2_gaps.json)
    if (!here.empty()) launch_tasks(here, /*staged=*/false, /*on_coord=*/b_.await_all);
  }

  // the update as its own launch (the unfused path)
  void launch_update(const UpdateSpec& u) {
    AggregateArgs a{};
    if (b_.n > kMaxAggregate) fail(MPA_ARGUMENT_ERROR, "aggregate: 0 <= nchunks <= %d", kMaxAggregate);
    a.chunks = b_.recvbuf;
    a.out = u.x;
    a.n = b_.n;
    a.elems = u.elems;
    a.stride = u.elems;
    a.eta = u.eta;
    a.update = 1;
    a.mirror = u.mirror;
    for (int64_t i = 0; i < b_.n; ++i) a.w[i] = u.w[size_t(i)];
    HIPCHECK(launch_aggregate(u.dtype, a, coord_));
  }

  bool fused_ok(const UpdateSpec& u, const std::vector<int64_t>& posted) const {
    const size_t es = u.dtype == MPA_F64 ? 8 : 4;
    if (b_.n > kMaxEpochChunks || int64_t(u.w.size()) != b_.n || b_.rl != size_t(u.elems) * es ||
        b_.sl != size_t(u.elems) * (u.msg_bf16 ? 2 : es) || b_.sendbuf != (u.msg_bf16 ? (const uint8_t*)u.mirror : (const uint8_t*)u.x))
      return false;
    size_t ndst = 0, ndoor = 0;
    for (int64_t rank : posted) {
      const bool remote = w_[size_t(rank - 1)].remote;
      ndst += remote ? 2 : 1;
      ndoor += remote ? 1 : 0;
    }
    return ndst <= size_t(kMaxEpochDst) && ndoor <= size_t(kMaxDoorbells);
  }

  // the epoch step can ride as the fused tail of the launch of `posted`: one batched
  // least-squares launch on the coordinator stream (local, undelayed, same shape, the
  // update's dtype), no doorbells, no bf16 mirror
  bool tail_fits(const std::vector<int64_t>& posted, const UpdateSpec& u) const {
    if (!fused_tail_ || posted.empty() || posted.size() > size_t(kMaxLsqTasks) || u.msg_bf16 || u.mirror) return false;
    int cp = -1;
    for (int64_t rank : posted) {
      const HipWorker& w = w_[size_t(rank - 1)];
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      if (w.remote || ts.kind != MPA_TASK_LSQ || !ts.delays_ns.empty() || ts.dtype != u.dtype) return false;
      const int c = lsq_cols_pad(ts.dtype, int(ts.cols));
      if (c > kLsqWideSlice) return false;  // wide rows: two launches, no fused tail
      if (cp >= 0 && c != cp) return false;
      cp = c;
    }
    return true;
  }

  // ONE epoch kernel: harvests [0, before) of `hv`, the update, harvests [before, end), the
  // dispatch copies of the posts (isendbuf slot; mailbox + doorbell for a remote worker)
  void emit_epoch(const std::vector<Harvest>& hv, size_t before, const std::vector<int64_t>& posted,
                  const UpdateSpec& u, hipStream_t s) {
    EpochArgs a = epoch_args(hv, before, posted, u);
    if (a.ndoor > 0) {
      a.ticket = ticket_;
      a.ticket_base = ticket_count_;
      ticket_count_ += uint32_t(epoch_grid(u.dtype, a));
    }
    if (timing_) {
      // the exchange this kernel performs over xGMI: messages into remote workers' slots
      // and replies read from their inboxes (mpa_comm_exchange_timing)
      double remote = 0;
      for (int64_t rank : posted)
        if (w_[size_t(rank - 1)].remote) remote += double(b_.sl);
      for (const Harvest& h : hv)
        if (w_[size_t(h.rank - 1)].remote) remote += double(b_.rl);
      XTimed xt{};
      {
        // the straggler timer thread takes events for its deferred launches too
        std::lock_guard<std::mutex> lk(tm_mu_);
        xt.start = take_event();
        xt.stop = take_event();
      }
      xt.remote_bytes = remote;
      HIPCHECK(hipEventRecord(xt.start, s));
      HIPCHECK(launch_epoch(u.dtype, a, s));
      HIPCHECK(hipEventRecord(xt.stop, s));
      xtimed_.push_back(xt);
      return;
    }
    HIPCHECK(launch_epoch(u.dtype, a, s));
  }

  // the arguments of one epoch step (no doorbell ticket yet)
  EpochArgs epoch_args(const std::vector<Harvest>& hv, size_t before, const std::vector<int64_t>& posted,
                       const UpdateSpec& u) const {
    EpochArgs a{};
    a.elems = u.elems;
    a.n = int(b_.n);
    a.update = 1;
    a.recv = b_.recvbuf;
    for (size_t k = 0; k < hv.size(); ++k) {
      const HipWorker& w = w_[size_t(hv[k].rank - 1)];
      const uint8_t* src = w.remote ? reply_src(w) : b_.irecvbuf + size_t(hv[k].slot) * b_.rl;
      (k < before ? a.hsrc : a.hsrc2)[hv[k].slot] = src;
    }
    for (int64_t i = 0; i < b_.n; ++i) a.w[i] = u.w[size_t(i)];
    a.eta = u.eta;
    a.x = u.x;
    a.mirror = u.mirror;
    a.msg_bf16 = u.msg_bf16 ? 1 : 0;
    for (int64_t rank : posted) {
      const HipWorker& w = w_[size_t(rank - 1)];
      a.dst[a.ndst++] = b_.isendbuf + size_t(w.slot) * b_.sl;
      if (w.remote) {
        a.dst[a.ndst++] = msg_dst(w);
        a.door[a.ndoor] = w.box_door_dev;
        a.doorval[a.ndoor++] = w.seq;
      }
    }
    return a;
  }

  // enqueue the next epoch of an await-all call (set_ahead), once per call, when this
  // call has posted every worker of the pool
  void maybe_ahead() {
    // an ahead epoch whose step already ran in the previous launch's fused tail must be
    // enqueued now: the descent loop that set it up guarantees it (anything else would apply
    // that update twice)
    auto skip = [this]() {
      if (tail_pending_) fail(MPA_ERROR, "fused tail: the epoch it prepared was not enqueued ahead");
    };
    if (ahead_left_ <= 0 || !b_.await_all || int64_t(call_posts_.size()) != b_.n || !held_.empty()) return skip();
    UpdateSpec& u = ahead_pred_;
    for (const auto& cp : call_posts_)
      if (w_[size_t(cp.rank - 1)].preposted) return skip();
    // the next epoch's posts equal this call's: same slots, same buffers; only workers
    // whose task starts as soon as its message lands (no injected delay, whose sleep
    // begins at delivery on the host timer)
    std::vector<int64_t> posted;
    for (const auto& cp : call_posts_) {
      const HipWorker& w = w_[size_t(cp.rank - 1)];
      const TaskSpec& ts = tasks_[size_t(cp.rank - 1)];
      if (!w.remote && ((ts.kind != MPA_TASK_LSQ && ts.kind != MPA_TASK_LSQ_BATCH) || !ts.delays_ns.empty())) return skip();
      posted.push_back(cp.rank);
    }
    if (!fused_ok(u, posted)) return skip();
    const bool more = ahead_left_ >= 2;  // the call after next enqueues another ahead epoch
    ahead_left_ = 0;
    // the replies of this call's remote tasks must have landed before the epoch kernel
    // reads them (local tasks are stream-ordered before it on the coordinator stream)
    std::vector<Harvest> hv;
    WaitWordsArgs ww{};
    ww.err = err_dev_;
    ww.spin_ticks = spin_ticks();
    for (const auto& cp : call_posts_) {
      HipWorker& w = w_[size_t(cp.rank - 1)];
      if (w.remote) {
        if (g_wait_value_ops) {
          HIPCHECK(hipStreamWaitValue64(coord_, region_->dev(&w.box->done), w.seq, hipStreamWaitValueGte, ~0ull));
        } else {
          if (ww.n == kMaxWaitWords) {
            HIPCHECK(launch_wait_words(ww, coord_));
            ww.n = 0;
          }
          ww.word[ww.n] = region_->dev(&w.box->done);
          ww.target[ww.n] = w.seq;
          ++ww.n;
        }
      }
      hv.push_back({cp.slot, cp.rank});
    }
    if (ww.n) HIPCHECK(launch_wait_words(ww, coord_));
    for (int64_t rank : posted) w_[size_t(rank - 1)].seq += 1;  // the ahead epoch's task numbers
    if (tail_pending_) tail_pending_ = false;  // this step ran in the previous launch's tail
    else emit_epoch(hv, hv.size(), posted, u, coord_);
    // Fused tail: at nwait == n every epoch's step is the same (harvest all n, weight 1 each,
    // re-post all n), so when another ahead epoch follows, THIS epoch's launch runs the next
    // step in its last workgroup and the next maybe_ahead enqueues only the launch
    if (more && tail_fits(posted, u)) {
      tail_args_ = epoch_args(hv, hv.size(), posted, u);
      tail_ranks_ = posted.size();
      tail_next_ = true;
      tail_pending_ = true;
    }
    launch_local(posted);
    if (tail_next_) fail(MPA_ERROR, "fused tail: no least-squares launch took it");
    for (int64_t rank : posted) {
      HipWorker& w = w_[size_t(rank - 1)];
      w.seq -= 1;  // the pool's view: its next post() takes the enqueued number
      w.preposted = true;
      w.preharvest = true;
    }
    ahead_bufs_ = b_;
    ahead_upd_ = u;
    ahead_update_ = true;
  }

  // ---- device-memory (xGMI) payload path (shm.hpp kPathDevice) ----
  // A fine-grained device buffer exported by a HIP IPC handle into `handle`; `state` tells
  // the other process whether it may open it.  Falls back to a plain allocation (state
  // kIpcFailed, payloads then go through the host mailbox) if fine-grained memory or IPC is
  // unavailable, or with MPA_XGMI=0.
  void* ipc_alloc(size_t bytes, char* handle, volatile uint32_t* state) {
    void* p = nullptr;
    if (xgmi_ && hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained) == hipSuccess) {
      hipIpcMemHandle_t h;
      if (hipIpcGetMemHandle(&h, p) == hipSuccess) {
        std::memcpy(handle, &h, sizeof(h));
        __atomic_store_n(state, kIpcOk, __ATOMIC_RELEASE);
        return p;
      }
      (void)hipGetLastError();
      std::fprintf(stderr, "[mpa] hipIpcGetMemHandle failed: worker payloads use the host mailbox\n");
      (void)hipFree(p);
      p = nullptr;
    }
    (void)hipGetLastError();
    HIPCHECK(hipMalloc(&p, bytes));
    __atomic_store_n(state, kIpcFailed, __ATOMIC_RELEASE);
    return p;
  }

  void* ipc_open(const char* handle, int peer_dev) {
    if (peer_dev != dev_) {
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, dev_, peer_dev) != hipSuccess || !can) {
        (void)hipGetLastError();
        return nullptr;
      }
      const hipError_t e = hipDeviceEnablePeerAccess(peer_dev, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
        (void)hipGetLastError();
        return nullptr;
      }
      (void)hipGetLastError();
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof(h));
    void* p = nullptr;
    if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    return p;
  }

  // coordinator, first post to a remote worker: once the server has exported its message
  // slot and opened our reply inbox, open its slot and fix the path for good
  void decide_path(int64_t rank) {
    HipWorker& w = w_[size_t(rank - 1)];
    BoxHeader* b = w.box;
    const auto t0 = Clock::now();
    for (uint64_t spins = 0; __atomic_load_n(&b->msg_ipc, __ATOMIC_ACQUIRE) == kIpcPending ||
                             __atomic_load_n(&b->reply_open, __ATOMIC_ACQUIRE) == kIpcPending;
         ++spins) {
      if ((spins & 0xFFF) == 0xFFF) watchdog(t0);
      __builtin_ia32_pause();
    }
    uint32_t mode = kPathHost;
    if (b->msg_ipc == kIpcOk && b->reply_open == kIpcOk && b->reply_ipc == kIpcOk) {
      w.peer_msg = static_cast<uint8_t*>(ipc_open(b->msg_handle, b->server_dev));
      if (w.peer_msg) mode = kPathDevice;
    }
    if (mode != kPathDevice && xgmi_)
      std::fprintf(stderr, "[mpa] worker %lld: device payload path unavailable, using the host mailbox\n",
                   (long long)rank);
    w.path_dev = mode == kPathDevice;
    w.path_known = true;
    __atomic_store_n(&b->mode, mode, __ATOMIC_RELEASE);
  }

  // server: open rank 0's reply inbox once it is exported; true once rank 0 fixed the path
  bool server_path(int64_t rank) {
    HipWorker& w = w_[size_t(rank - 1)];
    if (w.path_known) return true;
    BoxHeader* b = w.box;
    if (__atomic_load_n(&b->reply_open, __ATOMIC_ACQUIRE) == kIpcPending) {
      const uint32_t ri = __atomic_load_n(&b->reply_ipc, __ATOMIC_ACQUIRE);
      if (ri == kIpcPending) return false;
      if (ri == kIpcOk && b->msg_ipc == kIpcOk) w.peer_reply = static_cast<uint8_t*>(ipc_open(b->reply_handle, b->coord_dev));
      __atomic_store_n(&b->reply_open, w.peer_reply ? kIpcOk : kIpcFailed, __ATOMIC_RELEASE);
    }
    const uint32_t mode = __atomic_load_n(&b->mode, __ATOMIC_ACQUIRE);
    if (mode == kPathPending) return false;
    if (mode == kPathDevice && !w.peer_reply) fail(MPA_ERROR, "worker %lld: device path chosen without a reply inbox", (long long)rank);
    w.path_dev = mode == kPathDevice;
    w.path_known = true;
    return true;
  }

  // where rank 0 stores a remote worker's message / reads its reply
  uint8_t* msg_dst(const HipWorker& w) const { return w.path_dev ? w.peer_msg : w.box_msg_dev; }
  const uint8_t* reply_src(const HipWorker& w) const { return w.path_dev ? w.reply_inbox : w.box_reply_dev; }
  // where a served worker's task writes its reply
  uint8_t* reply_dst(const HipWorker& w) const { return w.path_dev ? w.peer_reply : w.box_reply_dev; }

  bool done(int64_t rank) const {
    const HipWorker& w = w_[size_t(rank - 1)];
    return __atomic_load_n(w.flag_host, __ATOMIC_ACQUIRE) >= w.seq && gate_open(rank, w.seq);
  }

  int64_t counter(const char* name) const override {
    const std::string k = name;
    if (k == "held") return n_held_;
    if (k == "held_joined") return n_held_joined_;
    if (k == "held_alone") return n_held_alone_;
    if (k == "gate_steps") return int64_t(gate_steps_taken());
    return -1;
  }

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

  void watchdog(Clock::time_point t0, bool timeout = true) {
    check_timer();
    const unsigned e = device_error();
    if (e) fail(MPA_DEVICE_ERROR, "device-side error word 0x%x (an in-kernel wait timed out)", e);
    for (auto& w : w_)
      if (w.stream) check_stream(w.stream);
    for (auto& s : launch_streams_) check_stream(s);
    if (timeout && timeout_s_ > 0 && std::chrono::duration<double>(Clock::now() - t0).count() > timeout_s_)
      fail(MPA_DEVICE_ERROR, "waited more than %.0f s for a worker (MPA_WAIT_TIMEOUT_S)", timeout_s_);
  }

  static void check_stream(hipStream_t s) {
    const hipError_t q = hipStreamQuery(s);
    if (q != hipSuccess && q != hipErrorNotReady) fail(MPA_DEVICE_ERROR, "worker stream error: %s", hipGetErrorString(q));
  }

  void check_task(int64_t rank, const TaskSpec& ts, size_t sl, size_t rl) {
    switch (ts.kind) {
      case MPA_TASK_ECHO: case MPA_TASK_KMAP1: case MPA_TASK_KMAP2: return;
      case MPA_TASK_LSQ: {
        const size_t es = ts.dtype == MPA_F64 ? 8 : 4;
        if (sl < size_t(ts.cols) * es)
          fail(MPA_DIMENSION_MISMATCH, "worker %lld (least squares, %lld columns) needs %zu bytes of sendbuf, got %zu",
               (long long)rank, (long long)ts.cols, size_t(ts.cols) * es, sl);
        if (rl < size_t(ts.cols) * es)
          fail(MPA_DIMENSION_MISMATCH, "worker %lld (least squares, %lld columns) replies %zu bytes, recv chunk is %zu",
               (long long)rank, (long long)ts.cols, size_t(ts.cols) * es, rl);
        if (role_ != SERVER &&
            ((reinterpret_cast<uintptr_t>(b_.isendbuf) | reinterpret_cast<uintptr_t>(b_.irecvbuf)) % es || sl % es || rl % es))
          fail(MPA_ARGUMENT_ERROR, "least-squares buffers must be %zu-byte aligned", es);
        return;
      }
      case MPA_TASK_LSQ_BATCH: {
        const size_t xb = size_t(ts.cols) * size_t(ts.k) * 2, gb = size_t(ts.cols) * size_t(ts.k) * 4;
        if (sl < xb)
          fail(MPA_DIMENSION_MISMATCH, "worker %lld (batched least squares, %lld x %lld bf16 X) needs %zu bytes of sendbuf, got %zu",
               (long long)rank, (long long)ts.cols, (long long)ts.k, xb, sl);
        if (rl < gb)
          fail(MPA_DIMENSION_MISMATCH, "worker %lld (batched least squares) replies %zu bytes (fp32 G), recv chunk is %zu",
               (long long)rank, gb, rl);
        if (role_ != SERVER &&
            ((reinterpret_cast<uintptr_t>(b_.isendbuf) | reinterpret_cast<uintptr_t>(b_.irecvbuf)) % 16 || sl % 16 || rl % 16))
          fail(MPA_ARGUMENT_ERROR, "batched least-squares buffers and messages must be 16-byte aligned");
        return;
      }
      default:
        fail(MPA_ERROR, "worker %lld has no task registered (mpa_comm_set_task_*)", (long long)rank);
    }
  }

  void prepare_lsq(int64_t rank, const TaskSpec& ts) {
    HipWorker& w = w_[size_t(rank - 1)];
    const int cp = lsq_cols_pad(ts.dtype, int(ts.cols));
    if (!cp) fail(MPA_ARGUMENT_ERROR, "least-squares worker: unsupported dtype/cols (%d, %lld)", ts.dtype, (long long)ts.cols);
    const int es = ts.dtype == MPA_F64 ? 8 : 4;
    const int E = 16 / es;
    if (ts.lda < ts.cols || ts.lda % E)
      fail(MPA_ARGUMENT_ERROR, "least-squares worker: lda (%lld) must be >= cols and a multiple of %d", (long long)ts.lda, E);
    if (reinterpret_cast<uintptr_t>(ts.A) % 16 || reinterpret_cast<uintptr_t>(ts.b) % size_t(es))
      fail(MPA_ARGUMENT_ERROR, "least-squares worker: A must be 16-byte aligned and b element aligned");
    if (role_ == SERVER && size_t(ts.cols) * size_t(es) > region_->max_msg())
      fail(MPA_DIMENSION_MISMATCH, "least-squares worker: %zu-byte messages exceed the mailbox", size_t(ts.cols) * es);
    const int cap = kSlabGridCap;
    // narrow: [grid][cols_pad] partials; wide: [slice][kLsqWideMaxGroups][2048] partials,
    // then the residual r (rows)
    const bool wide = cp > kLsqWideSlice;
    const size_t bytes = wide ? size_t(cp) * kLsqWideMaxGroups * size_t(es) + size_t(ts.rows + 64) * size_t(es)
                              : size_t(cap) * size_t(cp) * size_t(es);
    if (bytes > w.slab_bytes) {
      if (w.slab) {
        HIPCHECK(hipDeviceSynchronize());
        HIPCHECK(hipFree(w.slab));
      }
      w.slab = nullptr;
      HIPCHECK(hipMalloc(&w.slab, bytes));
      w.slab_bytes = bytes;
      w.slab_grid = cap;
    }
    if (wide && !w.wctr) {
      const size_t n = size_t(kLsqWideMaxCols / kLsqWideSlice + 1) * kLsqWideCtrPerSlice;
      HIPCHECK(hipMalloc(reinterpret_cast<void**>(&w.wctr), n * sizeof(uint32_t)));
      HIPCHECK(hipMemset(w.wctr, 0, n * sizeof(uint32_t)));
      HIPCHECK(hipDeviceSynchronize());
    }
  }

  // batched multi-iterate task: validate, size the residual scratch / partial slab
  void prepare_lsqb(int64_t rank, const TaskSpec& ts) {
    HipWorker& w = w_[size_t(rank - 1)];
    if (ts.k != kLsqbIterates)
      fail(MPA_ARGUMENT_ERROR, "batched least squares: %d iterates per message are supported, got %lld", kLsqbIterates,
           (long long)ts.k);
    if (ts.cols <= 0 || ts.cols % 32 || ts.cols > 256 * kLsqbMaxSlices)
      fail(MPA_ARGUMENT_ERROR, "batched least squares: cols (%lld) must be a positive multiple of 32, at most %d",
           (long long)ts.cols, 256 * kLsqbMaxSlices);
    if (ts.lda < ts.cols || ts.lda % 8)
      fail(MPA_ARGUMENT_ERROR, "batched least squares: lda (%lld) must be >= cols and a multiple of 8", (long long)ts.lda);
    if (reinterpret_cast<uintptr_t>(ts.A) % 16 || reinterpret_cast<uintptr_t>(ts.b) % 2)
      fail(MPA_ARGUMENT_ERROR, "batched least squares: A must be 16-byte aligned and B element aligned");
    if (ts.rows >= (int64_t(1) << 31)) fail(MPA_ARGUMENT_ERROR, "batched least squares: too many rows");
    if (role_ == SERVER && size_t(ts.cols) * size_t(ts.k) * 4 > region_->max_msg())
      fail(MPA_DIMENSION_MISMATCH, "batched least squares: %zu-byte replies exceed the mailbox",
           size_t(ts.cols) * size_t(ts.k) * 4);
    const size_t rows_pad = size_t((ts.rows + 255) / 256) * 256;
    const size_t rbytes = std::max<size_t>(rows_pad * size_t(kLsqbIterates) * 4, 256);
    if (rbytes > w.lsqb_R_bytes) {
      if (w.lsqb_R) HIPCHECK(hipFree(w.lsqb_R));
      w.lsqb_R = nullptr;
      HIPCHECK(hipMalloc(&w.lsqb_R, rbytes));
      w.lsqb_R_bytes = rbytes;
    }
    // pass-2 partials: [nrange][nslice][64 x 256 fp32]; nrange <= kLsqbRangeCap
    const size_t nslice = size_t((ts.cols + 255) / 256);
    const size_t sbytes = size_t(kLsqbRangeCap) * nslice * 256 * size_t(kLsqbIterates) * 4;
    if (sbytes > w.lsqb_slab_bytes) {
      if (w.lsqb_slab) HIPCHECK(hipFree(w.lsqb_slab));
      w.lsqb_slab = nullptr;
      HIPCHECK(hipMalloc(&w.lsqb_slab, sbytes));
      w.lsqb_slab_bytes = sbytes;
    }
    if (!w.lsqb_ctr) {
      HIPCHECK(hipMalloc(reinterpret_cast<void**>(&w.lsqb_ctr), sizeof(uint32_t) * (kLsqbMaxSlices + 1)));
      HIPCHECK(hipMemset(w.lsqb_ctr, 0, sizeof(uint32_t) * (kLsqbMaxSlices + 1)));
      HIPCHECK(hipDeviceSynchronize());
    }
    if (ts.cols <= kLsqpMaxCols && !w.lsqp_slab) {  // lsqp4 (and the measurement build's lsqp / lsqc)
      HIPCHECK(hipMalloc(&w.lsqp_slab, size_t(2) * kLsqpMaxGroups * 8 * 32 * 1024));
      const size_t nctr = size_t(2) * 8 * kLsqpCtrPerSlice + 8;  // + completions, lsqc ticket at +4
      HIPCHECK(hipMalloc(reinterpret_cast<void**>(&w.lsqp_ctr), sizeof(uint32_t) * nctr));
      HIPCHECK(hipMemset(w.lsqp_ctr, 0, sizeof(uint32_t) * nctr));
      // the column pairs' exchange ring (measurement build) is rewritten every kLsqcXR blocks:
      // in coarse-grained memory a reader's XCD L2 keeps serving its stale copy of a slot (sc1
      // loads bypass only L1), so the granules live in uncached device memory
      // (MPA_LSQC_XG=fine / coarse: A/B)
      if (MPA_MEASURE) {
        const size_t xg = size_t(kLsqpMaxGroups) * 2 * kLsqcXR * 4 * 64 * 4 * sizeof(unsigned long long);
        const char* e = measure_env("MPA_LSQC_XG");
        const unsigned fl = e && !std::strcmp(e, "fine") ? hipDeviceMallocFinegrained : hipDeviceMallocUncached;
        if (e && !std::strcmp(e, "coarse")) HIPCHECK(hipMalloc(reinterpret_cast<void**>(&w.lsqc_xg), xg));
        else HIPCHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&w.lsqc_xg), xg, fl));
        HIPCHECK(hipMemset(w.lsqc_xg, 0, xg));
      }
      HIPCHECK(hipDeviceSynchronize());
    }
    if (!MPA_MEASURE) return;  // the probe kernels' scratch (lsqq, lsqf): measurement build only
    if (ts.cols <= 2048 && !w.lsqq_ctr) {
      HIPCHECK(hipMalloc(reinterpret_cast<void**>(&w.lsqq_ctr), sizeof(uint32_t) * 8));
      HIPCHECK(hipMemset(w.lsqq_ctr, 0, sizeof(uint32_t) * 8));
    }
    if (ts.cols <= kLsqfMaxP * kLsqfSlice && !w.lsqf_x) {
      const size_t slots = size_t(kLsqfMaxGroups) * kLsqfXR * kLsqfMaxP;
      HIPCHECK(hipMalloc(&w.lsqf_x, slots * 4 * 64 * 16));
      HIPCHECK(hipMalloc(reinterpret_cast<void**>(&w.lsqf_flag), slots * sizeof(unsigned long long)));
      HIPCHECK(hipMemset(w.lsqf_flag, 0, slots * sizeof(unsigned long long)));
      // 8 slice / completion counters, then at byte 64 the per-XCD and arrival ticket words
      HIPCHECK(hipMalloc(reinterpret_cast<void**>(&w.lsqf_ctr), kLsqfCtrBytes));
      HIPCHECK(hipMemset(w.lsqf_ctr, 0, kLsqfCtrBytes));
      HIPCHECK(hipDeviceSynchronize());
    }
  }

  // workgroups per task in a least-squares launch of `ntasks` tasks
  int lsq_grid(const TaskSpec& ts, const HipWorker& w, int ntasks) const {
    static const int env_grid = [] { const char* e = measure_env("MPA_LSQ_GRID"); return e ? std::atoi(e) : 0; }();
    const int total = g_lsq_grid > 0 ? g_lsq_grid : env_grid > 0 ? env_grid : kDefaultLaunchGrid;
    const int rpw = lsq_rows_per_wave_iter(ts.dtype, int(ts.cols));
    const int64_t want = (ts.rows + 4 * rpw - 1) / (4 * rpw);
    int g = total / (ntasks > 0 ? ntasks : 1);
    if (g > want) g = int(want);
    if (g > w.slab_grid) g = w.slab_grid;
    if (g < 1) g = 1;
    return g;
  }

  // Tasks of one flush (coordinator) or one doorbell scan (server).  Least-squares tasks
  // without an injected delay run as ONE batched launch (per kernel variant, <=
  // kMaxLsqTasks each) on an idle launch stream; a task with a delay runs on its worker's
  // own stream behind a delay kernel, so a straggler never holds back another worker;
  // reference-test tasks (kmap/echo) run per worker.  `staged`: the message sits in a
  // mailbox and is first copied into the worker's device slot on the launch's stream.
  void launch_tasks(const std::vector<int64_t>& ranks, bool staged, bool on_coord = false) {
    std::vector<int64_t> batch;
    int batch_kind = -1, batch_dtype = -1, batch_cp = 0;
    hipStream_t bs = nullptr;
    bool ev_recorded = false;
    // the exchange that delivered the messages, as an event for other streams (once)
    auto after_exchange = [&](hipStream_t s) {
      if (!ev_recorded) {
        HIPCHECK(hipEventRecord(xfer_ev_, coord_));
        ev_recorded = true;
      }
      HIPCHECK(hipStreamWaitEvent(s, xfer_ev_, 0));
    };
    auto emit = [&]() {
      if (batch.empty()) return;
      bs = (on_coord || coord_batches_) && !staged ? coord_ : pick_launch_stream();
      if (staged) stage_in(batch, bs);
      else if (bs != coord_) after_exchange(bs);
      if (batch_kind == MPA_TASK_LSQ_BATCH) launch_lsqb_batch(batch, bs);
      else launch_lsq_batch(batch, batch_dtype, bs);
      batch.clear();
    };
    for (int64_t rank : ranks) {
      HipWorker& w = w_[size_t(rank - 1)];
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      int64_t delay = 0;
      if (!ts.delays_ns.empty()) delay = ts.delays_ns[size_t((int64_t(w.seq) - 1) % int64_t(ts.delays_ns.size()))];
      if ((ts.kind == MPA_TASK_LSQ || ts.kind == MPA_TASK_LSQ_BATCH) && delay == 0) {
        const int cp = ts.kind == MPA_TASK_LSQ ? lsq_cols_pad(ts.dtype, int(ts.cols)) : 0;
        if (!batch.empty() && (ts.kind != batch_kind || ts.dtype != batch_dtype || cp != batch_cp ||
                               batch.size() == size_t(kMaxLsqTasks)))
          emit();
        batch_kind = ts.kind;
        batch_dtype = ts.dtype;
        batch_cp = cp;
        batch.push_back(rank);
        continue;
      }
      // The message is delivered now (stream-ordered after the exchange / stage-in); a
      // delayed worker "sleeps" on the host timer and only then computes.
      if (staged) stage_in({rank}, worker_stream(w));
      else after_exchange(worker_stream(w));
      std::function<void()> go;
      if (ts.kind == MPA_TASK_LSQ) {
        double bytes = 0;
        const LsqBatch b = build_lsq_batch({rank}, ts.dtype, &bytes);
        const int cols = int(ts.cols), dt = ts.dtype;
        hipStream_t s = w.stream;
        go = [this, b, dt, cols, s, bytes]() { enqueue_lsq(b, dt, cols, s, bytes); };
      } else if (ts.kind == MPA_TASK_LSQ_BATCH) {
        double bytes = 0;
        const LsqbLaunch b = build_lsqb_batch({rank}, &bytes);
        hipStream_t s = w.stream;
        go = [this, b, s, bytes]() { enqueue_lsqb(b, s, bytes); };
      } else {
        KmapArgs a{};
        a.kind = ts.kind;
        a.rank = double(rank);
        a.x = w.x;
        a.sl = w.sl;
        a.out = w.out;
        a.rl = w.rl;
        a.pub = Publish{w.flag_dev, err_dev_, w.seq, spin_ticks()};
        hipStream_t s = w.stream;
        go = [a, s]() { HIPCHECK(launch_kmap(a, s)); };
      }
      if (delay > 0) defer(mono_ns() + uint64_t(delay), std::move(go));
      else go();
    }
    emit();
  }

  // ---- straggler emulation -------------------------------------------------------------
  // A worker with a delay schedule sleeps `delay` ns after its message is delivered and
  // then computes (the reference worker's `sleep(rand())` before its reply,
  // examples/iterative_example.jl:74).  The sleep is a host timer thread that launches the
  // task kernel when it is due, so a sleeping worker holds no GPU queue: kernels parked
  // in queues (a spinning delay kernel) made one straggler hold back another once the
  // process had more streams than the GPU maps hardware queues for.
  static uint64_t mono_ns() {
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count());
  }

  struct Deferred {
    uint64_t due;
    std::function<void()> go;
    bool operator<(const Deferred& o) const { return due > o.due; }  // min-heap on due
  };

  void defer(uint64_t due, std::function<void()> go) {
    std::lock_guard<std::mutex> lk(tmu_);
    if (!timer_.joinable()) {
      tstop_ = false;
      timer_ = std::thread([this]() { timer_loop(); });
    }
    deferred_.push_back(Deferred{due, std::move(go)});
    std::push_heap(deferred_.begin(), deferred_.end());
    tcv_.notify_all();
  }

  void timer_loop() {
    (void)hipSetDevice(dev_);
    std::unique_lock<std::mutex> lk(tmu_);
    for (;;) {
      if (tstop_) break;
      if (deferred_.empty()) {
        tidle_.notify_all();
        tcv_.wait(lk);
        continue;
      }
      const uint64_t due = deferred_.front().due, now = mono_ns();
      if (now + 200000 < due) {  // sleep to ~100 us before the deadline, then spin
        tcv_.wait_for(lk, std::chrono::nanoseconds(due - now - 100000));
        continue;
      }
      if (now < due) {
        lk.unlock();
        while (mono_ns() < due) __builtin_ia32_pause();
        lk.lock();
        continue;
      }
      std::pop_heap(deferred_.begin(), deferred_.end());
      Deferred d = std::move(deferred_.back());
      deferred_.pop_back();
      tbusy_ = true;
      lk.unlock();
      try {
        d.go();
      } catch (const Failure&) {
        std::lock_guard<std::mutex> g(tfail_mu_);
        if (tfail_msg_.empty()) tfail_msg_ = last_error();  // this thread's error text
        tfailed_.store(true, std::memory_order_release);
      }
      lk.lock();
      tbusy_ = false;
    }
  }

  // every deferred launch issued (shutdown)
  void drain_deferred() {
    std::unique_lock<std::mutex> lk(tmu_);
    if (!timer_.joinable()) return;
    tidle_.wait(lk, [this]() { return (deferred_.empty() && !tbusy_) || tstop_; });
  }

  // pending launches are dropped (the comm is being destroyed)
  void stop_timer() {
    {
      std::lock_guard<std::mutex> lk(tmu_);
      tstop_ = true;
      deferred_.clear();
      tcv_.notify_all();
      tidle_.notify_all();
    }
    if (timer_.joinable()) timer_.join();
  }

  void check_timer() {
    if (tfailed_.load(std::memory_order_acquire)) {
      std::lock_guard<std::mutex> g(tfail_mu_);
      fail(MPA_DEVICE_ERROR, "deferred task launch failed: %s", tfail_msg_.c_str());
    }
  }

  void stage_in(const std::vector<int64_t>& ranks, hipStream_t s) {
    ExchangeBuilder xb(ticket_, &ticket_count_, s);
    for (int64_t rank : ranks) {
      const HipWorker& w = w_[size_t(rank - 1)];
      if (w.path_dev) continue;  // rank 0 stored the message into the device slot itself
      if (debug_) {
        std::fprintf(stderr, "[mpa role %d] stage-in worker %lld: %zu bytes %p -> %p\n", int(role_), (long long)rank, w.sl,
                     (void*)w.box_msg_dev, (void*)w.xslot);
        describe("box msg", w.box_msg_dev);
        describe("xslot", w.xslot);
      }
      xb.copy(w.box_msg_dev, w.xslot, w.sl);
    }
    xb.launch();
    if (debug_) {
      const hipError_t e = hipStreamSynchronize(s);
      std::fprintf(stderr, "[mpa role %d] stage-in done: %s\n", int(role_), hipGetErrorString(e));
      std::fflush(stderr);
    }
  }

  // MPA_DEBUG=1: pointer attributes of everything handed to a kernel
  static void describe(const char* what, const void* p) {
    hipPointerAttribute_t at;
    const hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
      std::fprintf(stderr, "    %-8s %p: hipPointerGetAttributes failed: %s\n", what, p, hipGetErrorString(e));
      (void)hipGetLastError();
      return;
    }
    std::fprintf(stderr, "    %-8s %p: type %d device %d devptr %p hostptr %p\n", what, p, int(at.type), at.device,
                 at.devicePointer, at.hostPointer);
  }

  unsigned long long spin_ticks() const { return (unsigned long long)(timeout_s_ * rt_hz_); }

  // the worker's own stream (delayed tasks, pre-armed tasks), created on first use
  hipStream_t worker_stream(HipWorker& w) {
    if (!w.stream) w.stream = make_queue_stream(dev_);
    return w.stream;
  }
  // launch stream k (created on first use, up to kLaunchStreams)
  hipStream_t launch_stream(size_t k) {
    while (launch_streams_.size() <= k) launch_streams_.push_back(make_queue_stream(dev_));
    return launch_streams_[k];
  }

  // a launch stream with no pending work (so a batch never queues behind an unrelated
  // straggler's kernel); round-robin if every one is busy; a new one while fewer than
  // kLaunchStreams exist and all are busy
  hipStream_t pick_launch_stream() {
    if (launch_streams_.empty()) return launch_stream(0);
    const size_t m = launch_streams_.size();
    for (size_t k = 0; k < m; ++k) {
      const size_t j = (next_launch_ + k) % m;
      if (hipStreamQuery(launch_streams_[j]) == hipSuccess) {
        next_launch_ = (j + 1) % m;
        return launch_streams_[j];
      }
    }
    if (m < size_t(kLaunchStreams)) return launch_stream(m);
    hipStream_t s = launch_streams_[next_launch_];
    next_launch_ = (next_launch_ + 1) % m;
    return s;
  }

  void launch_lsq_batch(const std::vector<int64_t>& ranks, int dtype, hipStream_t s) {
    double bytes = 0;
    LsqBatch b = build_lsq_batch(ranks, dtype, &bytes);
    if (tail_next_) {  // maybe_ahead: this launch runs the next epoch's step (fused tail)
      if (s != coord_ || ranks.size() != tail_ranks_)
        fail(MPA_ERROR, "fused tail: the launch does not cover the epoch's %zu workers", tail_ranks_);
      b.tail = epoch_vec(dtype, tail_args_) ? 2 : 1;
      b.tail_ctr = tail_ctr_;
      b.ep = tail_args_;
      tail_next_ = false;
    }
    enqueue_lsq(b, dtype, int(tasks_[size_t(ranks[0] - 1)].cols), s, bytes);
  }

  // kernel arguments of one launch over `ranks`
  // `share`: the launch grid is divided as if this many tasks ran at once (concurrent
  // single-task launches of pre-armed workers)
  LsqBatch build_lsq_batch(const std::vector<int64_t>& ranks, int dtype, double* bytes_out, int share = 0) {
    LsqBatch b{};
    b.ntasks = int(ranks.size());
    const int split = share > b.ntasks ? share : b.ntasks;
    b.err = err_dev_;
    b.spin_ticks = spin_ticks();
    int blocks = 0;
    double bytes = 0;
    for (int k = 0; k < b.ntasks; ++k) {
      const int64_t rank = ranks[size_t(k)];
      HipWorker& w = w_[size_t(rank - 1)];
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      LsqTask& t = b.t[k];
      t.A = ts.A;
      t.b = ts.b;
      t.x = w.x;
      t.out = w.out;
      t.slab = w.slab;
      t.ctr = ctr_ + kLsqCtrPerTask * (rank - 1);
      t.flag = w.flag_dev;
      t.seq = w.seq;
      t.rows = ts.rows;
      t.lda = ts.lda;
      t.cols = int(ts.cols);
      t.grid = lsq_grid(ts, w, split);
      if (ts.cols > kLsqWideSlice) {  // wide rows: pass-1 workgroups, pass-2 row groups
        const int nslice = int((ts.cols + kLsqWideSlice - 1) / kLsqWideSlice);
        const int es = dtype == MPA_F64 ? 8 : 4;
        t.grid = int(std::max<int64_t>(1, std::min<int64_t>(kWideResidGrid / split, (ts.rows + 3) / 4)));
        t.grid2 = int(std::max<int64_t>(
            1, std::min<int64_t>({int64_t(kDefaultLaunchGrid) / split / nslice, int64_t(kLsqWideMaxGroups),
                                  (ts.rows + 7) / 8})));
        t.wctr = w.wctr;
        t.r = static_cast<uint8_t*>(w.slab) + size_t(nslice) * kLsqWideSlice * kLsqWideMaxGroups * size_t(es);
      }
      b.block0[k] = blocks;
      blocks += t.grid;
      const double es = dtype == MPA_F64 ? 8.0 : 4.0;
      bytes += es * (double(ts.rows) * double(ts.cols) + double(ts.rows) + 2.0 * double(ts.cols));
    }
    b.block0[b.ntasks] = blocks;
    *bytes_out = bytes;
    return b;
  }

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
  };

  // the iterate-halves single pass (lsqp_kernel.hip): the default for cols <= 2048
  // (MPA_LSQP=0 selects the two passes)
  bool lsqp_enabled(const std::vector<int64_t>& ranks) const {
    if (env_off("MPA_LSQP")) return false;
    for (int64_t rank : ranks) {
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      if (!w_[size_t(rank - 1)].lsqp_slab || ts.cols > kLsqpMaxCols) return false;
    }
    return !ranks.empty();
  }

  // column pairs (lsqc_kernel.hip): a row group of a task with more than 1024 columns is a
  // pair of workgroups (one each, 1024 columns and all 64 iterates), of a narrower task one
  // workgroup; 256 workgroups (one per CU) dealt over the tasks.  Row groups of at most
  // kLsqcMaxBlocks blocks (the tag's block field), else the iterate-halves kernel stays.
  static int lsqc_parts(int64_t cols) { return cols > kLsqcMemberCols ? 2 : 1; }
  int lsqc_groups(const TaskSpec& ts, int split, int k) const {
    constexpr int target = 256;
    const int per = target / split + (k < target % split ? 1 : 0);
    const int64_t nblocks = (ts.rows + 15) / 16;
    return int(std::max<int64_t>(1, std::min<int64_t>(std::min(per / lsqc_parts(ts.cols), kLsqpMaxGroups), nblocks)));
  }
  bool lsqc_fits(const std::vector<int64_t>& ranks, const LsqpBatch& b, int share) const {
    const int split = std::max(b.ntasks, share > 0 ? share : lsqb_share());
    for (size_t k = 0; k < ranks.size(); ++k) {
      const TaskSpec& ts = tasks_[size_t(ranks[k] - 1)];
      const int64_t nblocks = (ts.rows + 15) / 16;
      const int ng = lsqc_groups(ts, split, int(k));
      if ((nblocks + ng - 1) / ng > kLsqcMaxBlocks || !w_[size_t(ranks[k] - 1)].lsqc_xg) return false;
    }
    return true;
  }
  void build_lsqc(const std::vector<int64_t>& ranks, int share, LsqbLaunch& L) {
    LsqpBatch& b = L.halves;
    L.cpair = true;
    const int split = std::max(b.ntasks, share > 0 ? share : lsqb_share());
    int wgs = 0;
    for (int k = 0; k < b.ntasks; ++k) {
      const int64_t rank = ranks[size_t(k)];
      const HipWorker& w = w_[size_t(rank - 1)];
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      LsqpTask& t = b.t[k];
      t.xg = w.lsqc_xg;
      t.parts = lsqc_parts(ts.cols);
      b.grp0[k] = wgs;
      wgs += lsqc_groups(ts, split, k) * t.parts;
    }
    b.grp0[b.ntasks] = wgs;
    b.tick = w_[size_t(ranks[0] - 1)].lsqp_ctr + 2 * 8 * kLsqpCtrPerSlice + 4;
    b.pfd = lsqc_la_;  // lsqc: the phase-1 lookahead
    b.err = err_dev_;
    b.spin_ticks = spin_ticks();
  }

  // the iterate-quarter single pass (lsqq_kernel.hip): cols <= 2048 on every task
  bool lsqq_enabled(const std::vector<int64_t>& ranks) const {
    if (!MPA_MEASURE) return false;  // a probe kernel of the measurement build (make MEASURE=1)
    const char* e = measure_env("MPA_LSQQ");
    if (!e || *e != '1') return false;
    for (int64_t rank : ranks) {
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      if (!w_[size_t(rank - 1)].lsqq_ctr || ts.cols > 2048) return false;
    }
    return !ranks.empty();
  }

  bool lsqf_enabled(const std::vector<int64_t>& ranks) const {
    // measurement build, opt-in: the single-pass kernel is correct but, as measured
    // (DESIGN.md §10), slower than the two passes
    const char* e = measure_env("MPA_LSQF");
    if (!e || *e != '1') return false;
    int P = 0;
    for (int64_t rank : ranks) {
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      const HipWorker& w = w_[size_t(rank - 1)];
      const int p = int((ts.cols + kLsqfSlice - 1) / kLsqfSlice);
      if (!w.lsqf_x || p > kLsqfMaxP || (P && p != P)) return false;
      P = p;
    }
    return P > 0;
  }

  // kernel arguments over `ranks`; advances the workers' counter bases.  Algorithmic bytes
  // per task: A + B + X + G.
  // workers of this process with a batched least-squares task: a single-pass launch gives
  // each of its tasks the grid share of one of them, so that the launches of one epoch (all
  // fresh tasks, then a stale worker's re-dispatch, src/MPIAsyncPools.jl:177-184) run side
  // by side on disjoint CUs instead of the later one queueing behind a full-chip grid
  int lsqb_share() const {
    if (!lsqp_share_) return 1;
    int k = 0;
    for (int64_t r = 1; r <= nworkers_; ++r)
      k += w_[size_t(r - 1)].here && tasks_[size_t(r - 1)].kind == MPA_TASK_LSQ_BATCH;
    return k > 0 ? k : 1;
  }

  LsqbLaunch build_lsqb_batch(const std::vector<int64_t>& ranks, double* bytes_out, int share = 0) {
    LsqbLaunch L;
    double bytes = 0;
    for (int64_t rank : ranks) {
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      bytes += 2.0 * double(ts.rows) * double(ts.cols) + 2.0 * double(ts.rows) * double(ts.k) +
               2.0 * double(ts.cols) * double(ts.k) + 4.0 * double(ts.cols) * double(ts.k);
    }
    *bytes_out = bytes;
    if (lsqp_enabled(ranks) && !lsqf_enabled(ranks) && !lsqq_enabled(ranks)) {
      L.pair = true;
      L.pair8 = lsqp8_;
      LsqpBatch& b = L.halves;
      b.ntasks = int(ranks.size());
      b.pfd = lsqp_pfd_ >= 0 ? lsqp_pfd_ : (lsqp8_ ? 0 : 1);
      { const char* d = measure_env("MPA_LSQP_DBG"); b.dbg = d ? std::atoi(d) : 0; }
      // one workgroup per CU: 128 pairs (256 workgroups), dealt evenly over max(tasks,
      // share) tasks
      constexpr int target = 128;
      const int split = std::max(b.ntasks, share > 0 ? share : lsqb_share());
      int pairs = 0;
      for (int k = 0; k < b.ntasks; ++k) {
        const int64_t rank = ranks[size_t(k)];
        HipWorker& w = w_[size_t(rank - 1)];
        const TaskSpec& ts = tasks_[size_t(rank - 1)];
        LsqpTask& t = b.t[k];
        t.A = ts.A;
        t.B = ts.b;
        t.X = w.x;
        t.out = w.out;
        t.slab = w.lsqp_slab;
        t.ctr = w.lsqp_ctr;
        t.flag = w.flag_dev;
        t.seq = w.seq;
        t.rows = ts.rows;
        t.lda = ts.lda;
        t.cols = int(ts.cols);
        const int per = target / split + (k < target % split ? 1 : 0);
        const int64_t nblocks = (ts.rows + 15) / 16;
        const int ng = int(std::max<int64_t>(1, std::min<int64_t>(std::min(per, kLsqpMaxGroups), nblocks)));
        b.grp0[k] = pairs;
        pairs += ng;
      }
      b.grp0[b.ntasks] = pairs;
      if (lsqc_ && lsqc_fits(ranks, b, share)) build_lsqc(ranks, share, L);
      return L;
    }
    if (lsqq_enabled(ranks)) {
      L.quad = true;
      LsqqBatch& b = L.four;
      b.ntasks = int(ranks.size());
      { const char* d = measure_env("MPA_LSQQ_DBG"); b.dbg = d ? std::atoi(d) : 0; }
      // one 512-thread workgroup per CU: 64 quads (grid 256, a multiple of 32 so that each
      // quad's members share an XCD), dealt evenly over the tasks
      constexpr int target = 64;
      int groups = 0;
      for (int k = 0; k < b.ntasks; ++k) {
        const int64_t rank = ranks[size_t(k)];
        HipWorker& w = w_[size_t(rank - 1)];
        const TaskSpec& ts = tasks_[size_t(rank - 1)];
        LsqqTask& t = b.t[k];
        t.A = ts.A;
        t.B = ts.b;
        t.X = w.x;
        t.out = w.out;
        t.slab = w.lsqb_slab;
        t.ctr = w.lsqq_ctr;
        t.flag = w.flag_dev;
        t.seq = w.seq;
        t.rows = ts.rows;
        t.lda = ts.lda;
        t.cols = int(ts.cols);
        const int per = target / b.ntasks + (k < target % b.ntasks ? 1 : 0);
        const int64_t nblocks = (ts.rows + 15) / 16;
        const int ng = int(std::max<int64_t>(1, std::min<int64_t>(std::min(per, kLsqfMaxGroups), nblocks)));
        b.grp0[k] = groups;
        groups += ng;
      }
      b.grp0[b.ntasks] = groups;
      return L;
    }
    if (lsqf_enabled(ranks)) {
      L.fused = true;
      LsqfBatch& b = L.one;
      b.ntasks = int(ranks.size());
      b.err = err_dev_;
      b.spin_ticks = spin_ticks();
      // probe modes and the phase-1 lead: measurement build only (make MEASURE=1)
      { const char* d = measure_env("MPA_LSQF_DBG"); b.dbg = d ? std::atoi(d) : 0; }
      { const char* d = measure_env("MPA_LSQF_LAG"); b.lag = d ? std::atoi(d) : 4; }
      b.P = int((tasks_[size_t(ranks[0] - 1)].cols + kLsqfSlice - 1) / kLsqfSlice);
      // one workgroup per CU: groups of P, as many as keep the grid a multiple of 8 P (the
      // groups form inside an XCD, 8 XCDs), dealt evenly over the tasks
      const int target = std::max(1, (kLsqfGrid / b.P) / 8 * 8);
      HipWorker& w0 = w_[size_t(ranks[0] - 1)];
      b.tick = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(w0.lsqf_ctr) + 64);
      b.tag = uint32_t(w0.seq);
      int groups = 0;
      for (int k = 0; k < b.ntasks; ++k) {
        const int64_t rank = ranks[size_t(k)];
        HipWorker& w = w_[size_t(rank - 1)];
        const TaskSpec& ts = tasks_[size_t(rank - 1)];
        LsqfTask& t = b.t[k];
        t.A = ts.A;
        t.B = ts.b;
        t.X = w.x;
        t.out = w.out;
        t.xbuf = w.lsqf_x;
        t.xflag = w.lsqf_flag;
        t.slab = w.lsqb_slab;
        t.ctr = w.lsqf_ctr;
        t.flag = w.flag_dev;
        t.seq = w.seq;
        t.rows = ts.rows;
        t.lda = ts.lda;
        t.cols = int(ts.cols);
        const int64_t nblocks = (ts.rows + 15) / 16;
        const int per = target / b.ntasks + (k < target % b.ntasks ? 1 : 0);
        const int ng = int(std::max<int64_t>(1, std::min<int64_t>(std::min(per, kLsqfMaxGroups), nblocks)));
        t.sbase = w.lsqf_sbase;
        t.tbase = w.lsqf_tbase;
        w.lsqf_sbase += uint32_t(ng);
        w.lsqf_tbase += uint32_t(b.P);
        b.grp0[k] = groups;
        groups += ng;
      }
      b.grp0[b.ntasks] = groups;
      return L;
    }
    LsqbBatch& b = L.two;
    b.ntasks = int(ranks.size());
    b.err = err_dev_;
    b.spin_ticks = spin_ticks();
    int blocks1 = 0, blocks2 = 0;
    const int per1 = std::max(1, lsqb_grid(1) / b.ntasks), per2 = std::max(1, lsqb_grid(2) / b.ntasks);
    b.splitk = 1;
    for (int k = 0; k < b.ntasks; ++k)
      if (tasks_[size_t(ranks[size_t(k)] - 1)].cols > kLsqbSplitKCols) b.splitk = 0;
    for (int k = 0; k < b.ntasks; ++k) {
      const int64_t rank = ranks[size_t(k)];
      HipWorker& w = w_[size_t(rank - 1)];
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      LsqbTask& t = b.t[k];
      t.A = ts.A;
      t.B = ts.b;
      t.X = w.x;
      t.out = w.out;
      t.R = w.lsqb_R;
      t.slab = w.lsqb_slab;
      t.ctr = w.lsqb_ctr;
      t.flag = w.flag_dev;
      t.seq = w.seq;
      t.rows = ts.rows;
      t.lda = ts.lda;
      t.cols = int(ts.cols);
      const int64_t nblocks = b.splitk ? ((ts.rows + 31) / 32) * (32 / kLsqbSplitKRows) : (ts.rows + 255) / 256;
      t.grid1 = int(std::max<int64_t>(1, std::min<int64_t>(nblocks, per1)));
      t.nslice = int((ts.cols + 255) / 256);
      const int64_t ksteps = (ts.rows + 31) / 32;
      int64_t nr = per2 / t.nslice;
      if (nr >= 8) nr -= nr % 8;  // equal blk % 8 for the slices of a range (one XCD's L2)
      nr = std::max<int64_t>(1, std::min<int64_t>({nr, int64_t(kLsqbRangeCap), std::max<int64_t>(ksteps, 1)}));
      t.nrange = int(nr);
      t.sbase = w.lsqb_sbase;
      t.tbase = w.lsqb_tbase;
      w.lsqb_sbase += uint32_t(t.nrange);
      w.lsqb_tbase += uint32_t(t.nslice);
      b.block1[k] = blocks1;
      b.block2[k] = blocks2;
      blocks1 += t.grid1;
      blocks2 += t.nrange * t.nslice;
    }
    b.block1[b.ntasks] = blocks1;
    b.block2[b.ntasks] = blocks2;
    return L;
  }

  void enqueue_lsqb(const LsqbLaunch& b, hipStream_t s, double bytes, int64_t armed_rank = 0) {
    TimedLaunch tl{};
    const bool timed = timing_;
    if (timed) {
      std::lock_guard<std::mutex> lk(tm_mu_);
      tl.start = take_event();
      tl.stop = take_event();
      tl.bytes = bytes;
      tl.rank = armed_rank;
      HIPCHECK(hipEventRecord(tl.start, s));
    }
#if MPA_MEASURE
    HIPCHECK(b.pair ? (b.cpair ? launch_lsqc(b.halves, s) : b.pair8 ? launch_lsqp(b.halves, s) : launch_lsqp4(b.halves, s))
                    : b.quad ? launch_lsqq(b.four, s) : b.fused ? launch_lsqf(b.one, s) : launch_lsqb(b.two, s));
#else
    // the product carries the iterate-halves single pass and the two passes only
    HIPCHECK(b.pair ? launch_lsqp4(b.halves, s) : launch_lsqb(b.two, s));
#endif
    if (timed) {
      HIPCHECK(hipEventRecord(tl.stop, s));
      std::lock_guard<std::mutex> lk(tm_mu_);
      timed_.push_back(tl);
    }
  }

  // enqueue one least-squares launch on `s` (coordinator / server thread or timer thread)
  void enqueue_lsq(const LsqBatch& b, int dtype, int cols, hipStream_t s, double bytes, int64_t armed_rank = 0) {
    TimedLaunch tl{};
    const bool timed = timing_;
    if (timed) {
      std::lock_guard<std::mutex> lk(tm_mu_);
      tl.start = take_event();
      tl.stop = take_event();
      tl.bytes = bytes;
      tl.rank = armed_rank;
    }
    if (timed) HIPCHECK(hipEventRecord(tl.start, s));
    if (debug_) {
      for (int k = 0; k < b.ntasks; ++k) {
        const LsqTask& t = b.t[k];
        std::fprintf(stderr, "[mpa role %d] lsq task seq %llu grid %d A %p b %p x %p out %p slab %p ctr %p flag %p\n",
                     int(role_), t.seq, t.grid, t.A, t.b, t.x, t.out, t.slab, (void*)t.ctr, (void*)t.flag);
        describe("A", t.A);
        describe("x", t.x);
        describe("out", t.out);
        describe("flag", t.flag);
      }
      std::fflush(stderr);
    }
    HIPCHECK(launch_lsq(dtype, cols, b, s));
    if (debug_) {
      const hipError_t e = hipStreamSynchronize(s);
      std::fprintf(stderr, "[mpa role %d] lsq launch done: %s\n", int(role_), hipGetErrorString(e));
      std::fflush(stderr);
    }
    if (timed) {
      HIPCHECK(hipEventRecord(tl.stop, s));
      std::lock_guard<std::mutex> lk(tm_mu_);
      timed_.push_back(tl);
    }
  }

 public:
  // ---- kernel timing (HIP events around every least-squares launch) ----
  void set_timing(bool on) {
    if (!on) reap_timing(true);
    timing_ = on;
  }
  // launches, total kernel ms, total algorithmic bytes, and the ms during which at least
  // one timed launch was running (the union of their intervals: concurrent single-task
  // launches of delayed workers overlap) since the last call
  void timing(double out[4]) {
    reap_timing(true);
    std::sort(t_iv_.begin(), t_iv_.end());
    double busy = 0, hi = -1e300;
    for (const auto& iv : t_iv_) {
      if (iv.second <= hi) continue;
      busy += iv.second - (iv.first > hi ? iv.first : hi);
      hi = iv.second;
    }
    out[0] = double(t_launches_);
    out[1] = t_ms_;
    out[2] = t_bytes_;
    out[3] = busy;
    reap_xtiming();
    t_launches_ = 0;
    t_ms_ = 0;
    t_bytes_ = 0;
    t_iv_.clear();
    std::lock_guard<std::mutex> lk(tm_mu_);
    if (anchor_) event_pool_.push_back(anchor_);
    anchor_ = nullptr;
  }

 private:
  // epoch kernels timed since the last exchange_timing(): launches, ms, remote payload bytes
  struct XTimed {
    hipEvent_t start, stop;
    double remote_bytes;
  };
  std::vector<XTimed> xtimed_;
  double x_launches_ = 0, x_ms_ = 0, x_remote_ = 0;
  void reap_xtiming() {
    for (XTimed& xt : xtimed_) {
      HIPCHECK(hipEventSynchronize(xt.stop));
      float ms = 0;
      HIPCHECK(hipEventElapsedTime(&ms, xt.start, xt.stop));
      x_launches_ += 1;
      x_ms_ += ms;
      x_remote_ += xt.remote_bytes;
      std::lock_guard<std::mutex> lk(tm_mu_);
      event_pool_.push_back(xt.start);
      event_pool_.push_back(xt.stop);
    }
    xtimed_.clear();
  }

 public:
  void exchange_timing(double out[3]) {
    reap_xtiming();
    out[0] = x_launches_;
    out[1] = x_ms_;
    out[2] = x_remote_;
    x_launches_ = x_ms_ = x_remote_ = 0;
  }

 private:
  struct TimedLaunch {
    hipEvent_t start, stop;
    double bytes;
    int64_t rank;  // pre-armed launch of this worker (0: none)
    bool void_ = false;  // cancelled before it ran: not counted
  };

  // the pending timed launch armed for `rank` was cancelled
  void void_timing(int64_t rank) {
    std::lock_guard<std::mutex> lk(tm_mu_);
    for (auto it = timed_.rbegin(); it != timed_.rend(); ++it)
      if (it->rank == rank && !it->void_) {
        it->void_ = true;
        break;
      }
  }

  // caller holds tm_mu_ (event_pool_ is shared with the straggler timer thread)
  hipEvent_t take_event() {
    if (!event_pool_.empty()) {
      hipEvent_t e = event_pool_.back();
      event_pool_.pop_back();
      return e;
    }
    hipEvent_t e;
    HIPCHECK(hipEventCreate(&e));
    return e;
  }

  void reap_timing(bool block) {
    std::lock_guard<std::mutex> lk(tm_mu_);
    size_t keep = 0;
    for (size_t k = 0; k < timed_.size(); ++k) {
      TimedLaunch& tl = timed_[k];
      if (block) {
        HIPCHECK(hipEventSynchronize(tl.stop));
      } else if (hipEventQuery(tl.stop) != hipSuccess) {
        timed_[keep++] = tl;
        continue;
      }
      bool keep_start = false;
      if (!tl.void_) {
        float ms = 0, s0 = 0;
        HIPCHECK(hipEventElapsedTime(&ms, tl.start, tl.stop));
        if (!anchor_) {
          anchor_ = tl.start;  // interval origin of this timing window
          keep_start = true;
        } else {
          HIPCHECK(hipEventElapsedTime(&s0, anchor_, tl.start));
        }
        t_iv_.emplace_back(double(s0), double(s0) + double(ms));
        t_ms_ += ms;
        t_bytes_ += tl.bytes;
        t_launches_ += 1;
      }
      if (!keep_start) event_pool_.push_back(tl.start);
      event_pool_.push_back(tl.stop);
    }
    timed_.resize(keep);
  }

  Role role_ = SOLO;
  std::vector<HipWorker> w_;
  ShmRegion* region_ = nullptr;
  int my_rank_ = 0;
  int dev_ = 0;
  hipStream_t coord_ = nullptr;
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
  bool hold_ok_ = true;     // MPA_HOLD=0: a stale re-dispatch launches at once (flush_stale)
  bool hold_next_ = false;  // set while flush_stale() flushes
  bool may_hold_ = false;   // this call's wait completes without the held tasks (set_wait_hold)
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
  size_t tail_ranks_ = 0;
  EpochArgs tail_args_{};
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
  bool debug_ = false;
  int arm_mode_ = 0;
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
  std::atomic<bool> tfailed_{false};
  std::mutex tfail_mu_;
  std::string tfail_msg_;

 public:
  void init_ticket() {
    ticket_ = ctr_ + kLsqCtrPerTask * nworkers_;
    tail_ctr_ = ticket_ + 1;
  }
};

}  // namespace

Comm* make_hip_comm(int64_t nworkers, const int* devices) {
  HipComm* c = new HipComm(nworkers, devices, nullptr, 0, nullptr);
  c->init_ticket();
  return c;
}

Comm* make_dist_comm(int64_t nworkers, const int* placement, int my_rank, const char* shm_name, size_t max_msg) {
  if (!placement) fail(MPA_ARGUMENT_ERROR, "placement is NULL");
  if (!shm_name || !*shm_name) fail(MPA_ARGUMENT_ERROR, "shared memory name is empty");
  for (int64_t i = 0; i < nworkers; ++i)
    if (placement[i] < 0) fail(MPA_ARGUMENT_ERROR, "placement of worker %lld is negative", (long long)(i + 1));
  std::unique_ptr<ShmRegion> r(my_rank == 0 ? ShmRegion::create(shm_name, nworkers, max_msg)
                                            : ShmRegion::attach(shm_name));
  HipComm* c = new HipComm(nworkers, nullptr, placement, my_rank, r.get());
  r.release();
  c->init_ticket();
  return c;
}

void hip_set_stream(Comm* c, void* s) { static_cast<HipComm*>(c)->set_stream(static_cast<hipStream_t>(s)); }
void* hip_get_stream(Comm* c) { return static_cast<HipComm*>(c)->stream(); }
void hip_set_timing(Comm* c, bool on) { static_cast<HipComm*>(c)->set_timing(on); }
void hip_timing(Comm* c, double out[4]) { static_cast<HipComm*>(c)->timing(out); }
void hip_exchange_timing(Comm* c, double out[3]) { static_cast<HipComm*>(c)->exchange_timing(out); }
void hip_serve(Comm* c) { static_cast<HipComm*>(c)->serve(); }

namespace {
HipComm::UpdateSpec update_spec(int dtype, int64_t elems, const double* w, int64_t n, double eta, void* x,
                                void* mirror, bool msg_bf16) {
  HipComm::UpdateSpec u;
  u.dtype = dtype;
  u.elems = elems;
  u.w.assign(w, w + n);
  u.eta = eta;
  u.x = x;
  u.mirror = static_cast<uint16_t*>(mirror);
  u.msg_bf16 = msg_bf16;
  return u;
}
}  // namespace

void hip_set_defer_end(Comm* c, bool on) { static_cast<HipComm*>(c)->set_defer_end_flush(on); }
void hip_stage_update(Comm* c, int dtype, int64_t elems, const double* w, int64_t n, double eta, void* x, void* mirror,
                      bool msg_bf16) {
  static_cast<HipComm*>(c)->stage_update(update_spec(dtype, elems, w, n, eta, x, mirror, msg_bf16));
}
void hip_set_ahead(Comm* c, int64_t left, int dtype, int64_t elems, const double* w, int64_t n, double eta, void* x,
                   void* mirror, bool msg_bf16) {
  static_cast<HipComm*>(c)->set_ahead(left, update_spec(dtype, elems, w, n, eta, x, mirror, msg_bf16));
}
void hip_flush(Comm* c) { static_cast<HipComm*>(c)->flush(); }
int hip_payload_path(Comm* c, int64_t rank) { return static_cast<HipComm*>(c)->payload_path(rank); }
void hip_pause_servers(Comm* c) { static_cast<HipComm*>(c)->pause_servers(); }

}  // namespace mpa
