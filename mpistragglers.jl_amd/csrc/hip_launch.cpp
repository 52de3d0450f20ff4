// HipComm, task launches: registration-time scratch (prepare_*), batching the tasks of a
// flush into one launch per kernel, kernel arguments of the least-squares kernels (c1-c5),
// injected straggler delays (host timer thread, or a sleep kernel on the worker's stream),
// HIP-event timing, and
// the process-wide, capped set of CU-masked streams.
#include "hip_transport.hpp"

namespace mpa {

int g_lsq_grid = 0;  // mpa_tune("lsq_grid", G): workgroups per least-squares launch (0 = default)

// Process-wide set of CU-masked streams (each its own HSA queue).  Communicators come and go
// (tests create many), but the queues are a bounded hardware resource: once a device carries
// more queues than the scheduler maps at once, it time-slices them, and a launch on an
// unmapped queue waits up to ~10 ms for its turn -- also inside the launch call.  Measured
// (profiles/r04_queue_latency.txt, tools/probe_queue_latency.hip): launch -> visible of a
// one-wave kernel on a random idle queue, max 27 us with up to 20 CU-masked queues in the
// process, p99 8.4 ms with 24, 34 of 150 launches > 1 ms with 32; the gated kmap2_n9 replay
// ran within 1.5 ms of the oracle until a 24-worker comm grew the pool, then 578-643
// harvests were 1-25 ms late (r04_gated_stall.txt).  So the process holds at most
// queue_cap() of them per device (MPA_MAX_QUEUES, default 10, leaving room for the runtime's
// and torch's own); a comm returns its streams here, the next one reuses them, and past the
// cap workers share the least-used stream (a delayed worker then sleeps on a shared queue:
// stream_shared()).
// Past the cap a stream is only shared with streams of its own kind: a launch stream never
// carries a worker's (possibly sleeping, delayed) tasks, so a batch never queues behind an
// unrelated straggler, and a coordinator stream never carries tasks.
struct QueueStream {
  int device;
  hipStream_t s;
  int users;
  StreamKind kind;
  bool reserved;  // its CU mask leaves the reserved CUs out
};
std::mutex g_stream_mu;
std::vector<QueueStream> g_streams;
std::atomic<int> g_past_cap{0};

static int queue_cap() {
  static const int cap = [] {
    const char* e = std::getenv("MPA_MAX_QUEUES");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : kDefaultMaxQueues;
  }();
  return cap;
}

// The streams (and their HSA queues) are destroyed at process exit, before the HIP
// runtime's own teardown (atexit handlers run in reverse registration order, and the runtime
// registers its teardown when it is loaded, before the first stream here): a profiler that
// tears down while queues are still alive crashed in __cxa_finalize.
void destroy_pooled_streams() {
  std::lock_guard<std::mutex> lk(g_stream_mu);
  for (auto& q : g_streams) (void)hipStreamDestroy(q.s);
  g_streams.clear();
}

hipStream_t make_queue_stream(int device, StreamKind kind, bool reserved) {
  static const bool registered = (std::atexit(destroy_pooled_streams), true);
  (void)registered;
  reserved = reserved && kind != StreamKind::kCoord;
  std::lock_guard<std::mutex> lk(g_stream_mu);
  int have = 0;
  for (auto& q : g_streams)
    if (q.device == device) {
      if (q.users == 0 && q.reserved == reserved) {
        q.users = 1;
        q.kind = kind;
        return q.s;
      }
      ++have;
    }
  if (have >= queue_cap()) {  // share the least-used one of the same kind
    QueueStream* best = nullptr;
    for (auto& q : g_streams)
      if (q.device == device && q.kind == kind && q.reserved == reserved && (!best || q.users < best->users)) best = &q;
    if (best) {
      best->users += 1;
      return best->s;
    }
    // none of this kind yet: one more queue past the cap, said once (the cap is
    // no bound then; counter queues_past_cap)
    if (g_past_cap++ == 0)
      std::fprintf(stderr, "[mpa] %d CU-masked queues on device %d (MPA_MAX_QUEUES): one more for a stream kind "
                   "that has none yet\n", have, device);
  }
  hipDeviceProp_t p;
  HIPCHECK(hipGetDeviceProperties(&p, device));
  const int cus = p.multiProcessorCount;
  std::vector<uint32_t> mask(size_t((cus + 31) / 32), 0xFFFFFFFFu);
  if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
  if (reserved && cus >= 64) mask[0] &= ~((1u << kReservedCus) - 1u);  // CU 0 of each of the 8 XCDs
  hipStream_t s = nullptr;
  HIPCHECK(hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()));
  g_streams.push_back({device, s, 1, kind, reserved});
  return s;
}

int queues_past_cap() { return g_past_cap.load(); }

// The comm's own work is drained by its teardown (hipDeviceSynchronize in ~HipComm); a stream
// another live comm still uses is not synchronised here, so releasing never blocks on that
// comm's work.
void release_queue_stream(int device, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_stream_mu);
  for (auto& q : g_streams)
    if (q.device == device && q.s == s && q.users > 0) {
      if (q.users == 1) (void)hipStreamSynchronize(s);
      q.users -= 1;
      return;
    }
}

bool stream_shared(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_stream_mu);
  for (const auto& q : g_streams)
    if (q.s == s) return q.users > 1;
  return false;
}

int queue_streams(int device) {
  std::lock_guard<std::mutex> lk(g_stream_mu);
  int k = 0;
  for (const auto& q : g_streams) k += q.device == device;
  return k;
}

void HipComm::prepare_lsq(int64_t rank, const TaskSpec& ts) {
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

void HipComm::prepare_lsqb(int64_t rank, const TaskSpec& ts) {
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

int HipComm::lsq_grid(const TaskSpec& ts, const HipWorker& w, int ntasks) const {
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

void HipComm::launch_tasks(const std::vector<int64_t>& ranks, bool staged, bool on_coord) {
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
    MPA_HSTAMP('p', batch.front(), 0);
    bs = (on_coord || (coord_batches_ && !split_local_)) && !staged ? coord_ : pick_launch_stream();
    MPA_HSTAMP('q', batch.front(), 0);
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
    // delayed worker "sleeps" and only then computes: on the device, a deadline_kernel queued
    // ahead of the task on the worker's stream until the post time + the delay (device_delay_ok:
    // where no caller work on the NULL stream can wait behind it), or on the host timer thread,
    // which launches the task when it is due.
    hipStream_t s = worker_stream(w);
    const int64_t post_ns = int64_t(mono_ns());
    const bool on_device = delay > 0 && device_delay_ok(s);
    const int64_t sleep_ns = delay - (on_device ? deadline_lead_ns_ : delay_lead_ns_);
    const unsigned long long deadline = on_device && sleep_ns > 0 ? device_deadline(post_ns + sleep_ns) : 0;
    if (staged) stage_in({rank}, s);
    else after_exchange(s);
    std::function<void()> go;
    if (ts.kind == MPA_TASK_LSQ) {
      double bytes = 0;
      const LsqBatch b = build_lsq_batch({rank}, ts.dtype, &bytes);
      const int cols = int(ts.cols), dt = ts.dtype;
      go = [this, b, dt, cols, s, bytes]() { enqueue_lsq(b, dt, cols, s, bytes); };
    } else if (ts.kind == MPA_TASK_LSQ_BATCH) {
      double bytes = 0;
      const LsqbLaunch b = build_lsqb_batch({rank}, &bytes);
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
      a.pub_local = pub_local();
      int64_t* e = trace_entry(w);
      a.stamp = e ? reinterpret_cast<unsigned long long*>(e + kTStart) : nullptr;
      go = [a, s, e]() {
        if (e) e[kTCall] = int64_t(mono_ns());
        HIPCHECK(launch_kmap(a, s));
        if (e) e[kTRet] = int64_t(mono_ns());
      };
    }
    if (int64_t* e = trace_entry(w)) e[kTDue] = e[kTPost] + delay;
    // The oracle's worker replies exactly `delay` after its post; a task launched by the timer
    // takes ~30-40 us more (launch, the kernel, the completion word crossing the bus), one
    // queued behind a deadline ~8 us (its dispatch, the kernel, the word).  That overhead is
    // taken out of the sleep, or it would accumulate along every worker's chain of tasks: the
    // gated kmap2_n9 replay drifted 1.2-1.9 ms from the oracle's latencies by its 100th call
    // with 40 us per task (profiles/r04_gated_stall.txt).
    if (deadline) {
      HIPCHECK(launch_deadline(deadline, spin_ticks(), err_dev_, s));
      n_sleeps_ += 1;
      go();
    } else if (sleep_ns > 0) {
      defer(uint64_t(post_ns + sleep_ns), std::move(go));
    } else {
      go();
    }
  }
  emit();
}

// Device deadlines only where nothing can wait behind the sleeping wave but the worker's own
// task: a stream of its own (past the queue cap workers share one), and no caller work on the
// legacy NULL stream (HIP orders every NULL-stream command after all work queued on blocking
// streams, profiles/r04_delay_on_device.txt): a worker process (serve() runs no caller code),
// the native descent loop (its epochs are native code on the coordinator's own stream), or a
// caller on a stream of its own.  MPA_DELAY=timer / =device force either.
bool HipComm::device_delay_ok(hipStream_t s) const {
  if (delay_mode_ == 1 || stream_shared(s)) return false;
  if (delay_mode_ == 2) return true;
  return role_ == SERVER || defer_end_ || !caller_null_;
}

// host steady-clock ns -> device s_memrealtime ticks: the latest sample, and the rate measured
// between the first and the latest once they are a second apart (the two crystals drift by tens
// of ppm: tens of us per second).  The samples come from the first calibration
// (on_delays_changed) and the sampling thread (clock_loop); nothing here touches the GPU.
unsigned long long HipComm::device_deadline(int64_t host_ns) {
  std::lock_guard<std::mutex> g(ck_mu_);
  if (!ck_n0_) fail(MPA_ERROR, "device deadline without a clock calibration");
  const double rate = ck_n1_ - ck_n0_ >= kClockRateSpanNs ? double(ck_t1_ - ck_t0_) / double(ck_n1_ - ck_n0_) : rt_hz_ / 1e9;
  const double d = double(ck_t1_) + double(host_ns - ck_n1_) * rate;
  return d > 0 ? (unsigned long long)(d) : 0ull;
}

int64_t HipComm::clock_sample(hipStream_t s, int64_t* ticks, int64_t* ns) {
  if (!ck_probe_)
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&ck_probe_), 64, hipHostMallocCoherent | hipHostMallocMapped));
  __atomic_store_n(ck_probe_, 0ull, __ATOMIC_SEQ_CST);
  const int64_t t0 = int64_t(mono_ns());
  HIPCHECK(launch_clock_probe(reinterpret_cast<unsigned long long*>(ck_probe_), s));
  for (uint64_t spins = 0; __atomic_load_n(ck_probe_, __ATOMIC_ACQUIRE) == 0; ++spins) {
    if ((spins & 0xFFFF) == 0xFFFF && int64_t(mono_ns()) - t0 > 100000000) {  // 100 ms: a busy stream
      HIPCHECK(hipStreamSynchronize(s));
      return -1;
    }
    __builtin_ia32_pause();
  }
  const int64_t t1 = int64_t(mono_ns());
  *ticks = int64_t(__atomic_load_n(ck_probe_, __ATOMIC_ACQUIRE));
  *ns = t0 + (t1 - t0) / 2;
  return t1 - t0;
}

// The sampling thread of the clock map: one probe every 250 ms on a stream of its own, kept
// when its round trip is short (the midpoint is then within a few us of the probe's stamp).
void HipComm::clock_loop() {
  (void)hipSetDevice(dev_);
  std::unique_lock<std::mutex> lk(tmu_ck_);
  for (;;) {
    if (ck_cv_.wait_for(lk, std::chrono::nanoseconds(kClockRecalNs), [this]() { return ck_stop_; })) break;
    lk.unlock();
    int64_t t = 0, n = 0, rtt = -1;
    try {
      rtt = clock_sample(ck_stream_, &t, &n);
    } catch (...) {
      rtt = -1;  // (the map keeps its last sample)
    }
    if (rtt >= 0 && rtt <= kClockMaxRttNs) {
      std::lock_guard<std::mutex> g(ck_mu_);
      ck_t1_ = t;
      ck_n1_ = n;
      n_clock_samples_.fetch_add(1, std::memory_order_relaxed);
    }
    lk.lock();
  }
}

void HipComm::stop_clock() {
  {
    std::lock_guard<std::mutex> g(tmu_ck_);
    ck_stop_ = true;
  }
  ck_cv_.notify_all();
  if (ck_thread_.joinable()) ck_thread_.join();
}

void HipComm::defer(uint64_t due, std::function<void()> go) {
  std::lock_guard<std::mutex> lk(tmu_);
  if (!timer_.joinable()) {
    tstop_ = false;
    tstop_spin_.store(false, std::memory_order_release);
    timer_ = std::thread([this]() { timer_loop(); });
  }
  deferred_.push_back(Deferred{due, std::move(go)});
  std::push_heap(deferred_.begin(), deferred_.end());
  g_timer_pending.fetch_add(1, std::memory_order_relaxed);
  tfront_.store(deferred_.front().due, std::memory_order_release);
  tcv_.notify_all();
}

void HipComm::timer_loop() {
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
    // sleep to ~1 ms before the deadline, then spin: a condition-variable wake-up came up to
    // 0.6 ms late on a busy box (profiles/r04_gated_stall.txt, round 3's 100 us lead)
    if (now + kTimerSpinNs + 100000 < due) {
      tcv_.wait_for(lk, std::chrono::nanoseconds(due - now - kTimerSpinNs));
      continue;
    }
    if (now < due) {
      // spin with the lock released; a task deferred meanwhile with an earlier deadline moves
      // tfront_ below `due` and ends the spin (the loop then takes the new front), as does a stop
      lk.unlock();
      // yielding until the last 50 us (on a core it shares with the coordinator's wait neither
      // holds the other off), then pause-spinning: a yield that gives the core away for a
      // scheduler slice right at the deadline made the launch late
      uint64_t t;
      while ((t = mono_ns()) < due && tfront_.load(std::memory_order_acquire) >= due &&
             !tstop_spin_.load(std::memory_order_acquire)) {
        if (t + kTimerPauseNs < due) std::this_thread::yield();
        else __builtin_ia32_pause();
      }
      lk.lock();
      continue;
    }
    std::pop_heap(deferred_.begin(), deferred_.end());
    Deferred d = std::move(deferred_.back());
    deferred_.pop_back();
    g_timer_pending.fetch_sub(1, std::memory_order_relaxed);
    tfront_.store(deferred_.empty() ? ~0ull : deferred_.front().due, std::memory_order_release);
    tbusy_ = true;
    lk.unlock();
    const uint64_t t_go = mono_ns();
    if (t_go - d.due > 1000000) n_timer_late_.fetch_add(1, std::memory_order_relaxed);
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

void HipComm::stop_timer() {
  {
    std::lock_guard<std::mutex> lk(tmu_);
    tstop_ = true;
    tstop_spin_.store(true, std::memory_order_release);
    g_timer_pending.fetch_sub(int64_t(deferred_.size()), std::memory_order_relaxed);
    deferred_.clear();
    tfront_.store(~0ull, std::memory_order_release);
    tcv_.notify_all();
    tidle_.notify_all();
  }
  if (timer_.joinable()) timer_.join();
}

void HipComm::check_timer() {
  if (tfailed_.load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> g(tfail_mu_);
    fail(MPA_DEVICE_ERROR, "deferred task launch failed: %s", tfail_msg_.c_str());
  }
}

void HipComm::describe(const char* what, const void* p) {
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

hipStream_t HipComm::pick_launch_stream() {
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

void HipComm::launch_lsq_batch(const std::vector<int64_t>& ranks, int dtype, hipStream_t s) {
  double bytes = 0;
  LsqBatch b = build_lsq_batch(ranks, dtype, &bytes);
  if (tail_next_) {  // maybe_ahead: this launch runs the next epoch's step (fused tail)
    if (s != coord_ || ranks.size() != tail_ranks_)
      fail(MPA_ERROR, "fused tail: the launch does not cover the epoch's %zu workers", tail_ranks_);
    b.tail = epoch_vec(dtype, tail_args_) ? 2 : 1;
    b.tail_ctr = tail_ctr_;
    b.tail_nwait = tail_nwait_;
    for (int k = 0; k < tail_nwait_; ++k) {
      b.tail_word[k] = tail_word_[k];
      b.tail_target[k] = tail_target_[k];
    }
    b.ep = tail_args_;
    tail_next_ = false;
  } else if (head_next_) {  // flush: this launch runs this epoch's step first (fused head)
    if (s != coord_ || ranks.size() != head_ranks_ || batch_armed(b))
      fail(MPA_ERROR, "fused head: the launch does not cover the epoch's %zu workers", head_ranks_);
    b.head = epoch_vec(dtype, head_args_) ? 2 : 1;
    b.head_word = head_word_;
    b.head_token = next_head_token();
    b.ep = head_args_;
    head_next_ = false;
  }
  enqueue_lsq(b, dtype, int(tasks_[size_t(ranks[0] - 1)].cols), s, bytes);
}

LsqBatch HipComm::build_lsq_batch(const std::vector<int64_t>& ranks, int dtype, double* bytes_out, int share) {
  LsqBatch b{};
  b.ntasks = int(ranks.size());
  b.alone = here_count_ == 1 ? 1 : 0;
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
    t.flag2 = peer_done(w);
    t.seq = w.seq;
    t.rows = ts.rows;
    t.lda = ts.lda;
    t.cols = int(ts.cols);
    t.grid = lsq_grid(ts, w, split);
    t.pub_local = pub_local();
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

bool HipComm::lsqp_enabled(const std::vector<int64_t>& ranks) const {
  if (env_off("MPA_LSQP")) return false;
  for (int64_t rank : ranks) {
    const TaskSpec& ts = tasks_[size_t(rank - 1)];
    if (!w_[size_t(rank - 1)].lsqp_slab || ts.cols > kLsqpMaxCols) return false;
  }
  return !ranks.empty();
}

int HipComm::lsqc_groups(const TaskSpec& ts, int split, int k) const {
  constexpr int target = 256;
  const int per = target / split + (k < target % split ? 1 : 0);
  const int64_t nblocks = (ts.rows + 15) / 16;
  return int(std::max<int64_t>(1, std::min<int64_t>(std::min(per / lsqc_parts(ts.cols), kLsqpMaxGroups), nblocks)));
}

bool HipComm::lsqc_fits(const std::vector<int64_t>& ranks, const LsqpBatch& b, int share) const {
  const int split = std::max(b.ntasks, share > 0 ? share : lsqb_share());
  for (size_t k = 0; k < ranks.size(); ++k) {
    const TaskSpec& ts = tasks_[size_t(ranks[k] - 1)];
    const int64_t nblocks = (ts.rows + 15) / 16;
    const int ng = lsqc_groups(ts, split, int(k));
    if ((nblocks + ng - 1) / ng > kLsqcMaxBlocks || !w_[size_t(ranks[k] - 1)].lsqc_xg) return false;
  }
  return true;
}

void HipComm::build_lsqc(const std::vector<int64_t>& ranks, int share, LsqbLaunch& L) {
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

bool HipComm::lsqq_enabled(const std::vector<int64_t>& ranks) const {
  if (!MPA_MEASURE) return false;  // a probe kernel of the measurement build (make MEASURE=1)
  const char* e = measure_env("MPA_LSQQ");
  if (!e || *e != '1') return false;
  for (int64_t rank : ranks) {
    const TaskSpec& ts = tasks_[size_t(rank - 1)];
    if (!w_[size_t(rank - 1)].lsqq_ctr || ts.cols > 2048) return false;
  }
  return !ranks.empty();
}

bool HipComm::lsqf_enabled(const std::vector<int64_t>& ranks) const {
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

int HipComm::lsqb_share() const {
  if (!lsqp_share_) return 1;
  int k = 0;
  for (int64_t r = 1; r <= nworkers_; ++r)
    k += w_[size_t(r - 1)].here && tasks_[size_t(r - 1)].kind == MPA_TASK_LSQ_BATCH;
  return k > 0 ? k : 1;
}

HipComm::LsqbLaunch HipComm::build_lsqb_batch(const std::vector<int64_t>& ranks, double* bytes_out, int share) {
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
    b.err = err_dev_;  // the device-armed doorbell wait's error word and bound
    b.spin_ticks = spin_ticks();
    b.pfd = lsqp_pfd_ >= 0 ? lsqp_pfd_ : (lsqp8_ ? 0 : 1);
    { const char* d = measure_env("MPA_LSQP_DBG"); b.dbg = d ? std::atoi(d) : 0; }
    // one workgroup per CU: 128 pairs (256 workgroups), dealt evenly over max(tasks,
    // share) tasks; 120 (240) where the task streams leave one CU per XCD to the coordinator
    // (reserve_cus_: 31 CUs per XCD, a pair's two members on one XCD)
    const int target = reserve_cus_ ? 120 : 128;
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
      t.flag2 = peer_done(w);
      t.seq = w.seq;
      t.rows = ts.rows;
      t.lda = ts.lda;
      t.cols = int(ts.cols);
      t.pub_local = pub_local();
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
    t.flag2 = peer_done(w);
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

void HipComm::enqueue_lsqb(const LsqbLaunch& b, hipStream_t s, double bytes, int64_t armed_rank) {
  n_task_launches_.fetch_add(1, std::memory_order_relaxed);
  TimedLaunch tl{};
  const bool timed = sample_task(armed_rank);
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

void HipComm::enqueue_lsq(const LsqBatch& b, int dtype, int cols, hipStream_t s, double bytes, int64_t armed_rank,
                          bool untimed) {
  n_task_launches_.fetch_add(1, std::memory_order_relaxed);
  TimedLaunch tl{};
  // a pre-armed launch is never timed (it waits for the host inside); the launch pre-arming
  // skipped for the timing's sake always is
  bool timed = false;
  if (!untimed) {
    timed = time_next_ ? timing_.load() : sample_task(armed_rank);
    time_next_ = false;
  }
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
  {
    MPA_HPROF(kHpLaunch);
    MPA_HSTAMP('k', armed_rank, timed);
    HIPCHECK(launch_lsq(dtype, cols, b, s));
    MPA_HSTAMP('K', armed_rank, timed);
  }
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

void HipComm::timing(double out[4]) {
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

void HipComm::reap_xtiming() {
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

void HipComm::exchange_timing(double out[3]) {
  reap_xtiming();
  out[0] = x_launches_;
  out[1] = x_ms_;
  out[2] = x_remote_;
  x_launches_ = x_ms_ = x_remote_ = 0;
}

void HipComm::void_timing(int64_t rank) {
  std::lock_guard<std::mutex> lk(tm_mu_);
  for (auto it = timed_.rbegin(); it != timed_.rend(); ++it)
    if (it->rank == rank && !it->void_) {
      it->void_ = true;
      break;
    }
}

hipEvent_t HipComm::take_event() {
  if (!event_pool_.empty()) {
    hipEvent_t e = event_pool_.back();
    event_pool_.pop_back();
    return e;
  }
  hipEvent_t e;
  HIPCHECK(hipEventCreate(&e));
  return e;
}

void HipComm::reap_timing(bool block) {
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

}  // namespace mpa
