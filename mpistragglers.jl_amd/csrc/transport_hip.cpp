// HIP transport: the MPI point-to-point layer of MPIAsyncPools.jl replaced by device work.
//
//   MPI.Isend(isendbufs[i]) + MPI.Irecv!(irecvbufs[i])   (src/MPIAsyncPools.jl:137-138)
//     -> post(): deferred to flush(), where ONE exchange kernel on the coordinator stream
//        copies sendbuf into every posted slot of isendbuf (and performs the pending
//        harvest copies), one event is recorded, and each posted worker's stream waits
//        on it and runs [delay kernel] + task kernel.  The task kernel reads x from its
//        isendbuf slot and writes its reply into its irecvbuf chunk.
//   MPI.Test! / MPI.Waitany! / MPI.Waitall!               (:99, :161, :212)
//     -> loads of the worker's host-pinned completion word, which the task kernel's last
//        workgroup publishes with a system-scope release (no hipEventQuery, no sync call).
//   recvbufs[i] .= irecvbufs[i]                          (:108, :167, :216)
//     -> deferred and batched into the next exchange kernel on the coordinator stream,
//        which is ordered before any later re-post to that worker (the reference's
//        program order, :167 before :182-183).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "comm.hpp"
#include "kernels.hpp"

namespace mpa {

#define HIPCHECK(expr)                                                                  \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) fail(MPA_DEVICE_ERROR, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

int g_lsq_grid = 0;  // mpa_tune("lsq_grid", G): workgroups per least-squares task (0 = default)

namespace {

using Clock = std::chrono::steady_clock;

struct HipWorker {
  int device = 0;
  hipStream_t stream = nullptr;
  unsigned long long seq = 0;  // tasks posted
  // LSQ resources
  void* slab = nullptr;
  size_t slab_bytes = 0;
  int grid = 0;
  // per-post pointers
  int64_t slot = -1;
  const uint8_t* x = nullptr;
  uint8_t* out = nullptr;
  size_t sl = 0, rl = 0;
};

class HipComm final : public Comm {
 public:
  HipComm(int64_t n, const int* devices) : Comm(n), w_(size_t(n)) {
    HIPCHECK(hipGetDevice(&dev_));
    for (int64_t i = 0; i < n; ++i) {
      w_[size_t(i)].device = devices ? devices[i] : dev_;
      if (w_[size_t(i)].device != dev_)
        fail(MPA_ARGUMENT_ERROR, "worker %lld on device %d: workers on other devices than the coordinator's (%d) "
             "are served by per-device worker processes (DESIGN.md §Multi-GPU)", (long long)(i + 1),
             w_[size_t(i)].device, dev_);
    }
    for (auto& w : w_) HIPCHECK(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking));
    launch_streams_.resize(size_t(n < 2 ? 2 : n));
    for (auto& s : launch_streams_) HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&flags_), sizeof(unsigned long long) * size_t(n + 1),
                           hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(flags_, 0, sizeof(unsigned long long) * size_t(n + 1));
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&err_), 64, hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(err_, 0, 64);
    HIPCHECK(hipMalloc(&ctr_, sizeof(uint32_t) * 2 * size_t(n)));
    HIPCHECK(hipMemset(ctr_, 0, sizeof(uint32_t) * 2 * size_t(n)));
    HIPCHECK(hipEventCreateWithFlags(&xfer_ev_, hipEventDisableTiming));
    int khz = 0;
    HIPCHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_));
    rt_hz_ = khz > 0 ? double(khz) * 1e3 : 100e6;
    const char* g = std::getenv("MPA_LSQ_GRID");
    grid_max_ = g ? std::atoi(g) : 512;
    if (grid_max_ < 16) grid_max_ = 16;
    const char* t = std::getenv("MPA_WAIT_TIMEOUT_S");
    timeout_s_ = t ? std::atof(t) : 600.0;
    HIPCHECK(hipDeviceSynchronize());
  }

  ~HipComm() override {
    (void)hipDeviceSynchronize();
    for (auto& w : w_) {
      if (w.slab) (void)hipFree(w.slab);
      if (w.stream) (void)hipStreamDestroy(w.stream);
    }
    for (auto& s : launch_streams_) (void)hipStreamDestroy(s);
    for (auto& t : timed_) { (void)hipEventDestroy(t.start); (void)hipEventDestroy(t.stop); }
    for (auto e : event_pool_) (void)hipEventDestroy(e);
    if (ctr_) (void)hipFree(ctr_);
    if (flags_) (void)hipHostFree(flags_);
    if (err_) (void)hipHostFree(err_);
    if (xfer_ev_) (void)hipEventDestroy(xfer_ev_);
  }

  int transport() const override { return MPA_TRANSPORT_HIP; }
  void set_stream(hipStream_t s) { coord_ = s; }
  hipStream_t stream() const { return coord_; }
  double rt_hz() const { return rt_hz_; }

  void begin_call(const CallBufs& b) override { b_ = b; }

  void post(int64_t i, int64_t rank, int64_t tag) override {
    (void)tag;
    if (shutdown_) fail(MPA_ERROR, "comm has been shut down");
    HipWorker& w = w_[size_t(rank - 1)];
    const TaskSpec& ts = tasks_[size_t(rank - 1)];
    check_task(rank, ts, b_.sl, b_.rl);
    w.slot = i;
    w.x = b_.isendbuf + size_t(i) * b_.sl;
    w.out = b_.irecvbuf + size_t(i) * b_.rl;
    w.sl = b_.sl;
    w.rl = b_.rl;
    w.seq += 1;
    posts_.push_back(rank);
  }

  void harvest(int64_t i, int64_t rank) override {
    (void)rank;
    harv_.push_back(i);
  }

  bool test(int64_t i, int64_t rank) override {
    (void)i;
    return done(rank);
  }

  int64_t waitany(int64_t n, const int64_t* ranks, const uint8_t* live) override {
    bool any = false;
    for (int64_t i = 0; i < n; ++i) any |= live[i] != 0;
    if (!any) return -1;
    const auto t0 = Clock::now();
    for (uint64_t spins = 0;; ++spins) {
      for (int64_t i = 0; i < n; ++i)
        if (live[i] && done(ranks[i])) return i;
      if ((spins & 0xFFF) == 0xFFF) watchdog(t0);
      __builtin_ia32_pause();
    }
  }

  void waitall(int64_t n, const int64_t* ranks, const uint8_t* live) override {
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
    if (posts_.empty() && harv_.empty()) return;
    if (timing_) reap_timing(false);
    // the reference copies at dispatch/harvest time (:108, :130); here one kernel per flush
    size_t p = 0, h = 0;
    while (p < posts_.size() || h < harv_.size()) {
      ExchangeArgs ea{};
      ea.sendbuf = b_.sendbuf;
      ea.isendbuf = b_.isendbuf;
      ea.sl = b_.sl;
      ea.recvbuf = b_.recvbuf;
      ea.irecvbuf = b_.irecvbuf;
      ea.rl = b_.rl;
      for (; p < posts_.size() && ea.npost < kMaxExchangeItems; ++p)
        ea.post[ea.npost++] = int16_t(w_[size_t(posts_[p] - 1)].slot);
      for (; h < harv_.size() && ea.nharv < kMaxExchangeItems; ++h) ea.harv[ea.nharv++] = int16_t(harv_[h]);
      constexpr uint64_t kPart = 64 * 1024;
      ea.ppart = kPart;
      ea.hpart = kPart;
      ea.bpp = int((b_.sl + kPart - 1) / kPart);
      ea.bph = int((b_.rl + kPart - 1) / kPart);
      if (ea.bpp == 0) ea.npost = 0;
      if (ea.bph == 0) ea.nharv = 0;
      HIPCHECK(launch_exchange(ea, coord_));
    }
    harv_.clear();
    if (posts_.empty()) return;
    HIPCHECK(hipEventRecord(xfer_ev_, coord_));
    launch_posts();
    posts_.clear();
  }

  void end_call() override { flush(); }

  uint64_t now_ns() override {
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count());
  }

  int64_t tasks_done(int64_t rank) override {
    return int64_t(__atomic_load_n(&flags_[rank - 1], __ATOMIC_ACQUIRE));
  }

  void shutdown() override {
    const auto t0 = Clock::now();
    for (int64_t r = 1; r <= nworkers_; ++r)
      for (uint64_t spins = 0; !done(r); ++spins) {
        if ((spins & 0xFFF) == 0xFFF) watchdog(t0);
        __builtin_ia32_pause();
      }
    for (auto& w : w_) HIPCHECK(hipStreamSynchronize(w.stream));
    for (auto& s : launch_streams_) HIPCHECK(hipStreamSynchronize(s));
    shutdown_ = true;
  }

  void on_task_changed(int64_t rank) override {
    HipWorker& w = w_[size_t(rank - 1)];
    if (w.seq != uint64_t(tasks_done(rank)))
      fail(MPA_ERROR, "cannot change the task of worker %lld while it has an outstanding request", (long long)rank);
    const TaskSpec& ts = tasks_[size_t(rank - 1)];
    if (ts.kind == MPA_TASK_LSQ) prepare_lsq(rank, ts);
  }

  unsigned device_error() const { return __atomic_load_n(err_, __ATOMIC_ACQUIRE); }

 private:
  bool done(int64_t rank) const {
    return __atomic_load_n(&flags_[rank - 1], __ATOMIC_ACQUIRE) >= w_[size_t(rank - 1)].seq;
  }

  void watchdog(Clock::time_point t0) {
    const unsigned e = device_error();
    if (e) fail(MPA_DEVICE_ERROR, "device-side error word 0x%x (in-kernel wait timed out)", e);
    for (auto& w : w_) check_stream(w.stream);
    for (auto& s : launch_streams_) check_stream(s);
    if (timeout_s_ > 0 && std::chrono::duration<double>(Clock::now() - t0).count() > timeout_s_)
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
        if ((reinterpret_cast<uintptr_t>(b_.isendbuf) | reinterpret_cast<uintptr_t>(b_.irecvbuf)) % es ||
            sl % es || rl % es)
          fail(MPA_ARGUMENT_ERROR, "least-squares buffers must be %zu-byte aligned", es);
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
    const int rpw = lsq_rows_per_wave_iter(ts.dtype, int(ts.cols));
    const int R = lsq_reducers(ts.dtype, int(ts.cols));
    int64_t want = (ts.rows + 4 * rpw - 1) / (4 * rpw);
    const int gmax = g_lsq_grid > 0 ? g_lsq_grid : grid_max_;
    int grid = int(want < gmax ? want : gmax);
    if (grid < R) grid = R;
    const size_t bytes = size_t(grid) * size_t(cp) * size_t(es);
    if (bytes > w.slab_bytes) {
      if (w.slab) HIPCHECK(hipFree(w.slab));
      HIPCHECK(hipMalloc(&w.slab, bytes));
      w.slab_bytes = bytes;
    }
    w.grid = grid;
  }

  // Posts of one flush: least-squares tasks without an injected delay run as ONE batched
  // launch (per kernel variant, <= kMaxLsqTasks each) on an idle launch stream; a task
  // with a delay runs on its worker's own stream behind a delay kernel, so a straggler
  // never holds back another worker; reference-test tasks (kmap/echo) run per worker.
  void launch_posts() {
    std::vector<int64_t> batch;
    int batch_dtype = -1, batch_cp = 0;
    auto emit = [&](hipStream_t s) {
      if (batch.empty()) return;
      launch_lsq_batch(batch, batch_dtype, s);
      batch.clear();
    };
    for (int64_t rank : posts_) {
      HipWorker& w = w_[size_t(rank - 1)];
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      int64_t delay = 0;
      if (!ts.delays_ns.empty()) delay = ts.delays_ns[size_t((int64_t(w.seq) - 1) % int64_t(ts.delays_ns.size()))];
      if (ts.kind == MPA_TASK_LSQ && delay == 0) {
        const int cp = lsq_cols_pad(ts.dtype, int(ts.cols));
        if (!batch.empty() && (ts.dtype != batch_dtype || cp != batch_cp || batch.size() == size_t(kMaxLsqTasks)))
          emit(pick_launch_stream());
        batch_dtype = ts.dtype;
        batch_cp = cp;
        batch.push_back(rank);
        continue;
      }
      HIPCHECK(hipStreamWaitEvent(w.stream, xfer_ev_, 0));
      if (delay > 0) HIPCHECK(launch_delay((unsigned long long)(double(delay) * 1e-9 * rt_hz_), w.stream));
      if (ts.kind == MPA_TASK_LSQ) {
        std::vector<int64_t> one{rank};
        launch_lsq_batch(one, ts.dtype, w.stream, /*waited=*/true);
      } else {
        KmapArgs a{};
        a.kind = ts.kind;
        a.rank = double(rank);
        a.x = w.x;
        a.sl = w.sl;
        a.out = w.out;
        a.rl = w.rl;
        a.pub = Publish{&flags_[rank - 1], err_, w.seq, spin_ticks()};
        HIPCHECK(launch_kmap(a, w.stream));
      }
    }
    emit(pick_launch_stream());
  }

  unsigned long long spin_ticks() const { return (unsigned long long)(timeout_s_ * rt_hz_); }

  // a launch stream with no pending work (so a batch never queues behind an unrelated
  // straggler's kernel); round-robin if every one is busy
  hipStream_t pick_launch_stream() {
    const size_t m = launch_streams_.size();
    for (size_t k = 0; k < m; ++k) {
      const size_t j = (next_launch_ + k) % m;
      if (hipStreamQuery(launch_streams_[j]) == hipSuccess) {
        next_launch_ = (j + 1) % m;
        return launch_streams_[j];
      }
    }
    hipStream_t s = launch_streams_[next_launch_];
    next_launch_ = (next_launch_ + 1) % m;
    return s;
  }

  void launch_lsq_batch(const std::vector<int64_t>& ranks, int dtype, hipStream_t s, bool waited = false) {
    LsqBatch b{};
    b.ntasks = int(ranks.size());
    b.err = err_;
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
      t.ctr = ctr_ + 2 * (rank - 1);
      t.flag = &flags_[rank - 1];
      t.seq = w.seq;
      t.rows = ts.rows;
      t.lda = ts.lda;
      t.cols = int(ts.cols);
      t.grid = w.grid;
      b.block0[k] = blocks;
      blocks += w.grid;
      const double es = dtype == MPA_F64 ? 8.0 : 4.0;
      bytes += es * (double(ts.rows) * double(ts.cols) + double(ts.rows) + 2.0 * double(ts.cols));
    }
    b.block0[b.ntasks] = blocks;
    if (!waited) HIPCHECK(hipStreamWaitEvent(s, xfer_ev_, 0));
    TimedLaunch tl{};
    if (timing_) {
      tl.start = take_event();
      tl.stop = take_event();
      tl.bytes = bytes;
      HIPCHECK(hipEventRecord(tl.start, s));
    }
    HIPCHECK(launch_lsq(dtype, int(tasks_[size_t(ranks[0] - 1)].cols), b, s));
    if (timing_) {
      HIPCHECK(hipEventRecord(tl.stop, s));
      timed_.push_back(tl);
    }
  }

 public:
  // ---- kernel timing (HIP events around every least-squares launch) ----
  void set_timing(bool on) {
    if (!on) reap_timing(true);
    timing_ = on;
  }
  // launches, total kernel ms, total algorithmic bytes since the last call
  void timing(double out[3]) {
    reap_timing(true);
    out[0] = double(t_launches_);
    out[1] = t_ms_;
    out[2] = t_bytes_;
    t_launches_ = 0;
    t_ms_ = 0;
    t_bytes_ = 0;
  }

 private:
  struct TimedLaunch {
    hipEvent_t start, stop;
    double bytes;
  };

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
    size_t keep = 0;
    for (size_t k = 0; k < timed_.size(); ++k) {
      TimedLaunch& tl = timed_[k];
      if (block) HIPCHECK(hipEventSynchronize(tl.stop));
      else if (hipEventQuery(tl.stop) != hipSuccess) { timed_[keep++] = tl; continue; }
      float ms = 0;
      HIPCHECK(hipEventElapsedTime(&ms, tl.start, tl.stop));
      t_ms_ += ms;
      t_bytes_ += tl.bytes;
      t_launches_ += 1;
      event_pool_.push_back(tl.start);
      event_pool_.push_back(tl.stop);
    }
    timed_.resize(keep);
  }

  bool timing_ = false;
  std::vector<TimedLaunch> timed_;
  std::vector<hipEvent_t> event_pool_;
  int64_t t_launches_ = 0;
  double t_ms_ = 0, t_bytes_ = 0;
  std::vector<hipStream_t> launch_streams_;
  size_t next_launch_ = 0;

  int dev_ = 0;
  hipStream_t coord_ = nullptr;
  std::vector<HipWorker> w_;
  unsigned long long* flags_ = nullptr;
  unsigned* err_ = nullptr;
  uint32_t* ctr_ = nullptr;
  hipEvent_t xfer_ev_ = nullptr;
  double rt_hz_ = 100e6;
  int grid_max_ = 512;
  double timeout_s_ = 600.0;
  std::vector<int64_t> posts_, harv_;
  CallBufs b_;
};

}  // namespace

Comm* make_hip_comm(int64_t nworkers, const int* devices) { return new HipComm(nworkers, devices); }
void hip_set_stream(Comm* c, void* s) { static_cast<HipComm*>(c)->set_stream(static_cast<hipStream_t>(s)); }
void* hip_get_stream(Comm* c) { return static_cast<HipComm*>(c)->stream(); }
void hip_set_timing(Comm* c, bool on) { static_cast<HipComm*>(c)->set_timing(on); }
void hip_timing(Comm* c, double out[3]) { static_cast<HipComm*>(c)->timing(out); }

}  // namespace mpa
