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
#include "hip_transport.hpp"

#include <time.h>
#include <unistd.h>

namespace mpa {
#if MPA_MEASURE
HostProf g_hprof;

namespace {
struct HostStamp {
  char kind;
  int64_t a, b;
  int64_t t;
};
constexpr size_t kHostStamps = size_t(1) << 20;
std::vector<HostStamp>* g_hstamp = nullptr;
std::atomic<size_t> g_hstamp_n{0};
const char* g_hstamp_dir = nullptr;
void dump_host_stamps() {
  if (!g_hstamp) return;
  char path[512];
  std::snprintf(path, sizeof path, "%s/%d.txt", g_hstamp_dir, int(getpid()));
  if (FILE* f = std::fopen(path, "w")) {
    const size_t n = std::min(g_hstamp_n.load(), kHostStamps);
    for (size_t k = 0; k < n; ++k) {
      const HostStamp& h = (*g_hstamp)[k];
      std::fprintf(f, "%c %lld %lld %lld\n", h.kind, (long long)h.a, (long long)h.b, (long long)h.t);
    }
    std::fclose(f);
  }
}
}  // namespace

void host_stamp(char kind, int64_t a, int64_t b) {
  static const bool on = [] {
    g_hstamp_dir = std::getenv("MPA_HOST_STAMP");
    if (!g_hstamp_dir || !*g_hstamp_dir) return false;
    g_hstamp = new std::vector<HostStamp>(kHostStamps);
    std::atexit(dump_host_stamps);
    return true;
  }();
  if (!on) return;
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  const size_t k = g_hstamp_n.fetch_add(1, std::memory_order_relaxed);
  if (k < kHostStamps) (*g_hstamp)[k] = {kind, a, b, int64_t(ts.tv_sec) * 1000000000 + ts.tv_nsec};
}
#endif

// rank 0 waits for remote completions of a launched-ahead epoch with one wait_words_kernel
// (default) or, MPA_WAIT_VALUE_OPS=1 (measurement build), one hipStreamWaitValue64 per remote worker
const bool g_wait_value_ops = [] { const char* e = measure_env("MPA_WAIT_VALUE_OPS"); return e && *e == '1'; }();

HipComm::HipComm(int64_t n, const int* devices, const int* placement, int my_rank, ShmRegion* region)
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
  // two cancel words per worker (armed tasks s and s + 1), then the door_cas scratch word
  HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&cancel_), sizeof(unsigned long long) * size_t(2 * n + 1),
                         hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(cancel_, 0, sizeof(unsigned long long) * size_t(2 * n + 1));
  xgmi_ = !env_off("MPA_XGMI");
  done_dev_ = !env_off("MPA_DONE_DEV");
  // per-task tree counters, then the doorbell ticket and the fused-tail counter
  HIPCHECK(hipMalloc(&ctr_, sizeof(uint32_t) * (kLsqCtrPerTask * size_t(n) + 3)));
  HIPCHECK(hipMemset(ctr_, 0, sizeof(uint32_t) * (kLsqCtrPerTask * size_t(n) + 3)));
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
      // the message slot, then the worker's device doorbell word (device-armed tasks wait on it)
      w.xslot = static_cast<uint8_t*>(ipc_alloc(door_off() + 256, w.box->msg_handle, &w.box->msg_ipc));
      HIPCHECK(hipMemset(w.xslot + door_off(), 0, 256));
      w.cancel_host = &cancel_[2 * (r - 1)];
      w.cancel_dev = &cancel_[2 * (r - 1)];
    } else if (w.remote) {
      w.flag_host = &w.box->done;
      w.box->coord_dev = dev_;
      // the reply inbox, then the device copy of the worker's completion word (publish_peer)
      w.reply_inbox = static_cast<uint8_t*>(ipc_alloc(done_off() + 256, w.box->reply_handle, &w.box->reply_ipc));
      HIPCHECK(hipMemset(w.reply_inbox + done_off(), 0, 256));
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
  here_count_ = here_count;
  bool any_remote = false, coord_gpu = false;
  for (const auto& w : w_) {
    any_remote |= w.remote;
    if (role_ == SERVER && w.here && w.box) coord_gpu |= w.box->coord_dev == dev_;
  }
  split_local_ = role_ == COORD && any_remote && !env_off("MPA_SPLIT_LOCAL");
  // (opt-in, MPA_RESERVE_CUS=1: on the one-GPU rehearsal the reserved CUs cost c5 at N = 2 a
  // third of its rate -- 84 against 128 it/s, r06k -- while the split alone already brought the
  // epoch step from 236-356 us to 16 us; on the node it is unmeasured)
  const char* rc = std::getenv("MPA_RESERVE_CUS");
  reserve_cus_ = ((role_ == COORD && any_remote) || (role_ == SERVER && coord_gpu)) && rc && *rc == '1';
  const char* eager = measure_env("MPA_EAGER_STREAMS");
  if (eager && *eager == '1') {
    for (auto& w : w_)
      if (w.here) worker_stream(w);
    launch_stream(kLaunchStreams - 1);
  } else if (role_ == SERVER && here_count > 1) {
    launch_stream(kLaunchStreams - 1);
  }
  // the coordinator's own stream, in place of the NULL stream (set_stream)
  if (role_ != SERVER && !env_off("MPA_OWN_COORD")) coord_ = own_coord_ = make_queue_stream(dev_, StreamKind::kCoord);
  HIPCHECK(hipEventCreateWithFlags(&xfer_ev_, hipEventDisableTiming));
  HIPCHECK(hipEventCreateWithFlags(&switch_ev_, hipEventDisableTiming));
  int khz = 0;
  HIPCHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_));
  rt_hz_ = khz > 0 ? double(khz) * 1e3 : 100e6;
  const char* t = std::getenv("MPA_WAIT_TIMEOUT_S");
  timeout_s_ = t ? std::atof(t) : 600.0;
  // device-armed server tasks (hip_server.cpp): 0 never, 1 every eligible worker, 2 (default)
  // where a process serves one worker
  const char* arm = std::getenv("MPA_ARM");
  arm_mode_ = arm && *arm == '0' ? 0 : arm && *arm == '1' ? 1 : 2;
  const char* ad = std::getenv("MPA_ARM_DEPTH");
  arm_depth_env_ = ad && (*ad == '1' || *ad == '2') ? *ad - '0' : 0;
  // injected straggler delays: the host timer (default) or a sleep kernel ahead of the task on
  // an unshared worker stream (MPA_DELAY=device); the launch overhead taken out of each sleep
  const char* dl = std::getenv("MPA_DELAY");
  delay_mode_ = dl && !std::strcmp(dl, "timer") ? 1 : dl && !std::strcmp(dl, "device") ? 2 : 0;
  const char* lead = std::getenv("MPA_DELAY_LEAD_NS");
  if (lead) delay_lead_ns_ = std::atoll(lead);
  const char* dlead = std::getenv("MPA_DEADLINE_LEAD_NS");
  if (dlead) deadline_lead_ns_ = std::atoll(dlead);
  // how an armed task waits: one wave ahead of it (default) or every workgroup in-kernel
  const char* aw = std::getenv("MPA_ARM_WAIT");
  arm_wave_ = !(aw && !std::strcmp(aw, "kernel"));
  // measurement build: the in-kernel wait also on a GPU rank 0 uses (the one-GPU rehearsal of
  // the node's path; the product refuses it there)
  const char* af = measure_env("MPA_ARM_WAIT_FORCE");
  arm_force_ = af && *af == '1';
  const char* cb = measure_env("MPA_COORD_BATCH");
  coord_batches_ = !(cb && *cb == '0');
  fused_tail_ = !env_off("MPA_TAIL");
  fused_head_ = !env_off("MPA_HEAD");
  prearm_ = fused_head_ && !env_off("MPA_PREARM");
  defer_ok_ = !env_off("MPA_DEFER");
  msg_wt_ = !env_off("MPA_MSG_WT");
  pub_local_ = !env_off("MPA_PUB_LOCAL");
  pre_same_ = !env_off("MPA_PRESAME");
  HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&pre_mb_), sizeof(PreMailbox), hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(static_cast<void*>(pre_mb_), 0, sizeof(PreMailbox));
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
#if MPA_MEASURE
  if (const char* hs = measure_env("MPA_HEAD_STAMP"); hs && *hs == '1') head_stamp_reset();
#endif
  const char* dbg = std::getenv("MPA_DEBUG");
  debug_ = dbg && *dbg == '1';
  if (debug_ && region_) {
    std::fprintf(stderr, "[mpa role %d rank %d] shm header %p (device %p)\n", int(role_), my_rank_,
                 (void*)region_->header(), (void*)region_->dev(region_->header()));
    describe("shm", region_->dev(region_->header()));
  }
  HIPCHECK(hipDeviceSynchronize());
}

HipComm::~HipComm() {
  try {
    release_held();
    disarm_all();
  } catch (...) {
  }
  stop_timer();
  stop_clock();
  (void)hipDeviceSynchronize();
#if MPA_MEASURE
  if (const char* d = measure_env("MPA_LSQF_DBG"); d && (std::atoi(d) & 16)) lsqf_prof_dump();
  if (const char* d = measure_env("MPA_LSQP4_CLOCK"); d && *d == '1') lsqp4_clock_dump();
  if (const char* d = measure_env("MPA_LSQ_STAMP"); d && *d == '1') lsq_stamp_dump();
  if (const char* d = measure_env("MPA_HEAD_STAMP"); d && *d == '1') head_stamp_dump();
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
  if (own_coord_) release_queue_stream(dev_, own_coord_);
  for (auto& t : timed_) {
    (void)hipEventDestroy(t.start);
    (void)hipEventDestroy(t.stop);
  }
  for (auto e : event_pool_) (void)hipEventDestroy(e);
  if (ctr_) (void)hipFree(ctr_);
  if (flags_) (void)hipHostFree(flags_);
  if (err_) (void)hipHostFree(err_);
  if (cancel_) (void)hipHostFree(cancel_);
  if (trace_) (void)hipHostFree(trace_);
  if (clock_probe_) (void)hipHostFree(clock_probe_);
  if (ck_probe_) (void)hipHostFree(ck_probe_);
  if (ck_stream_) (void)hipStreamDestroy(ck_stream_);
  if (pre_mb_) {
    cancel_pre();
    (void)hipStreamSynchronize(coord_);  // the cancelled launch has left before its mailbox goes
    (void)hipHostFree(pre_mb_);
  }
  if (xfer_ev_) (void)hipEventDestroy(xfer_ev_);
  if (switch_ev_) (void)hipEventDestroy(switch_ev_);
  delete region_;
}

void HipComm::check_buffers(const CallBufs& b) {
  const void* ps[4] = {b.sl ? b.sendbuf : nullptr, b.rl ? b.recvbuf : nullptr, b.sl ? b.isendbuf : nullptr,
                       b.rl ? b.irecvbuf : nullptr};
  if (std::equal(ps, ps + 4, checked_bufs_)) return;
  static const char* names[4] = {"sendbuf", "recvbuf", "isendbuf", "irecvbuf"};
  for (int k = 0; k < 4; ++k) {
    if (!ps[k]) continue;
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, ps[k]);
    if (e != hipSuccess || a.type == hipMemoryTypeUnregistered) {
      (void)hipGetLastError();
      fail(MPA_ARGUMENT_ERROR, "%s is host memory the GPU cannot address: a device comm takes device buffers", names[k]);
    }
  }
  std::copy(ps, ps + 4, checked_bufs_);
}

void HipComm::post(int64_t i, int64_t rank, int64_t tag) {
  MPA_HPROF(kHpPost);
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
    trace_post(w, rank);
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
  trace_post(w, rank);
  posts_.push_back(rank);
}

void HipComm::harvest(int64_t i, int64_t rank) {
  MPA_HPROF(kHpHarvest);
  HipWorker& w = w_[size_t(rank - 1)];
  if (int64_t* e = trace_entry(w)) e[kTHarvest] = int64_t(mono_ns());
  if (w.preharvest) {  // already in the epoch kernel enqueued ahead
    w.preharvest = false;
    return;
  }
  harv_.push_back({i, rank});
}

int64_t HipComm::waitany(int64_t n, const int64_t* ranks, const uint8_t* live) {
  MPA_HPROF(kHpWaitany);
  bool any = false;
  for (int64_t i = 0; i < n; ++i) any |= live[i] != 0;
  if (!any) return -1;
  if (!held_.empty() && !may_hold_) {  // the wait would block: held launches go first
    for (int64_t i = 0; i < n; ++i)
      if (live[i] && done(ranks[i])) return i;
    release_held();
  }
  const auto t0 = Clock::now();
  PoliteSpin poll;
  for (uint64_t spins = 0;; ++spins) {
    for (int64_t i = 0; i < n; ++i)
      if (live[i] && done(ranks[i])) {
        MPA_HSTAMP('R', ranks[i], w_[size_t(ranks[i] - 1)].seq);
        return i;
      }
    if ((spins & 0xFFF) == 0xFFF) watchdog(t0);
    poll();
  }
}

void HipComm::waitall(int64_t n, const int64_t* ranks, const uint8_t* live) {
  cancel_pre();
  release_held();
  const auto t0 = Clock::now();
  for (int64_t i = 0; i < n; ++i) {
    if (!live[i]) continue;
    PoliteSpin poll;
    for (uint64_t spins = 0; !done(ranks[i]); ++spins) {
      if ((spins & 0xFFF) == 0xFFF) watchdog(t0);
      poll();
    }
  }
}

void HipComm::flush() {
  MPA_HPROF(kHpFlush);
  if (pre_active_ && pre_consume()) return;  // the pre-armed launch runs this epoch
  if (defer_stale()) return;                 // held re-dispatches: nothing to launch yet
  cancel_pre();
  if (!stale_deferred_.empty() && (!has_update_ || !fused_ok(upd_, posts_) || !deferred_fit(upd_))) run_deferred();
  if (posts_.empty() && harv_.empty() && !has_update_) {
    maybe_ahead();
    return;
  }
  if (timing_) reap_timing(false);
  if (has_update_ && fused_ok(upd_, posts_)) {
    if (head_fits(posts_, upd_)) {  // the step runs at the head of the task launch
      head_args_ = epoch_args(harv_, harv_before_, posts_, upd_);
      head_next_ = true;
      last_head_ranks_ = launch_ranks();
      head_ranks_ = last_head_ranks_.size();
      ++n_head_;
    } else {
      emit_epoch(harv_, harv_before_, posts_, upd_, coord_);
    }
    stale_deferred_.clear();  // the step carried them
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
        xb.reserve(2, 2);
        xb.copy(b_.sendbuf, slot, b_.sl);
        xb.copy(b_.sendbuf, msg_dst(w), b_.sl);
        xb.door(w.box_door_dev, w.seq);
        if (w.path_dev) xb.door(peer_door(w), w.seq);
      } else {
        xb.copy(b_.sendbuf, slot, b_.sl);
      }
    }
    xb.launch();
  }
  has_update_ = false;
  harv_.clear();
  const bool headed = !last_head_ranks_.empty();
  const int hdtype = upd_.dtype;
  launch_local(posts_);
  if (head_next_) fail(MPA_ERROR, "fused head: no least-squares launch took it");
  posts_.clear();
  maybe_ahead();
  if (headed) maybe_prearm(hdtype);
  last_head_ranks_.clear();
}

// The next epoch, enqueued now behind this one (pre-armed): only in the descent loop at
// nwait < n (launch-ahead and the fused tail cover nwait = n), right after a fused-head launch
// of the whole pool, and not for the one launch in `timing_period_` that the timing samples.
void HipComm::maybe_prearm(int dtype) {
  MPA_HPROF(kHpPrearm);
  if (!prearm_ || !prearm_loop_ || !defer_end_ || b_.await_all || gated() || role_ != SOLO || pre_active_ || !held_.empty())
    return;
  if (timing_ && timing_period_ > 1 && ++pre_count_ % timing_period_ == 0) {
    time_next_ = true;
    return;
  }
  if (timing_ && timing_period_ <= 1) return;  // every launch timed: none pre-armed
  const std::vector<int64_t>& ranks = last_head_ranks_;
  for (int64_t rank : ranks) w_[size_t(rank - 1)].seq += 1;  // the tasks of the next epoch
  double bytes = 0;
  LsqBatch b = build_lsq_batch(ranks, dtype, &bytes);
  pre_seq_.clear();
  pre_x_.clear();
  pre_out_.clear();
  for (int64_t rank : ranks) {
    HipWorker& w = w_[size_t(rank - 1)];
    pre_seq_.push_back(w.seq);
    pre_x_.push_back(w.x);
    pre_out_.push_back(w.out);
    w.seq -= 1;
  }
  pre_vec_ = epoch_vec(dtype, head_args_);
  b.head = (pre_vec_ ? 2 : 1) | kHeadPrearmed;
  b.head_word = head_word_;
  b.head_token = next_head_token();
  b.pre_go = &pre_mb_->go;
  b.pre_ep = &pre_mb_->ep;
  b.ep = head_args_;  // the prediction: this epoch's step again (c1's steady state)
  pre_pred_ = head_args_;
  b.pre_token = ++pre_token_;
  pre_ranks_ = ranks;
  pre_active_ = true;
  enqueue_lsq(b, dtype, int(tasks_[size_t(ranks[0] - 1)].cols), coord_, bytes, 0, /*untimed=*/true);
}

// This flush is the epoch the pre-armed launch was enqueued for: the same workers posted to
// the same slots with the task numbers it carries, a fused-head step.  Its arguments go to
// the mailbox, then the go word (release: the launch reads them after it).
bool HipComm::pre_consume() {
  MPA_HPROF(kHpPreConsume);
  const std::vector<int64_t> ranks = launch_ranks();
  if (!has_update_ || ranks != pre_ranks_ || hold_next_ || !fused_ok(upd_, posts_) || !head_fits(posts_, upd_) ||
      !deferred_fit(upd_))
    return false;
  for (size_t k = 0; k < ranks.size(); ++k) {
    const HipWorker& w = w_[size_t(ranks[k] - 1)];
    if (w.seq != pre_seq_[k] || w.x != pre_x_[k] || w.out != pre_out_[k]) return false;
  }
  EpochArgs ea = epoch_args(harv_, harv_before_, posts_, upd_);
  if (ea.ndoor != 0 || epoch_vec(upd_.dtype, ea) != pre_vec_) return false;
  if (pre_same_ && std::memcmp(&ea, &pre_pred_, sizeof ea) == 0) {
    __atomic_store_n(&pre_mb_->go, pre_token_ | kPreSame, __ATOMIC_RELEASE);  // as predicted
    ++n_pre_same_;
  } else {
    std::memcpy(static_cast<void*>(&pre_mb_->ep), &ea, sizeof ea);
    __atomic_store_n(&pre_mb_->go, pre_token_, __ATOMIC_RELEASE);
  }
  pre_active_ = false;
  head_args_ = ea;
  ++n_head_;
  ++n_prearmed_;
  const int dtype = upd_.dtype;
  has_update_ = false;
  harv_.clear();
  stale_deferred_.clear();
  n_held_joined_ += int64_t(held_.size());
  held_.clear();
  last_head_ranks_ = ranks;
  posts_.clear();
  maybe_prearm(dtype);
  last_head_ranks_.clear();
  return true;
}

void HipComm::release_held() {
  cancel_pre();
  run_deferred();  // their messages first
  if (held_.empty()) return;
  std::vector<int64_t> h;
  h.swap(held_);
  n_held_alone_ += int64_t(h.size());
  launch_tasks(h, /*staged=*/false);
}

void HipComm::stage_update(const UpdateSpec& u) {
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

void HipComm::shutdown() {
  cancel_pre();
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

void HipComm::on_task_changed(int64_t rank) {
  cancel_pre();
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

// A delay schedule registered for a worker of this process: its stream now (a stream is never
// created inside a timed schedule), and the first host <-> device clock sample behind device
// deadlines (best of 16 round trips on that idle stream).
void HipComm::on_delays_changed(int64_t rank) {
  HipWorker& w = w_[size_t(rank - 1)];
  if (!w.here || tasks_[size_t(rank - 1)].delays_ns.empty()) return;
  hipStream_t s = worker_stream(w);
  if (ck_thread_.joinable()) return;
  int64_t best = INT64_MAX;
  for (int k = 0; k < 16; ++k) {
    int64_t t = 0, n = 0;
    const int64_t rtt = clock_sample(s, &t, &n);
    if (rtt >= 0 && rtt < best) {
      best = rtt;
      ck_t0_ = ck_t1_ = t;
      ck_n0_ = ck_n1_ = n;
    }
  }
  if (best == INT64_MAX) fail(MPA_DEVICE_ERROR, "clock calibration: no probe landed");
  n_clock_samples_ = 1;
  HIPCHECK(hipStreamCreateWithFlags(&ck_stream_, hipStreamNonBlocking));
  ck_stop_ = false;
  ck_thread_ = std::thread([this]() { clock_loop(); });
}

void HipComm::launch_local(const std::vector<int64_t>& posted) {
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
  if (!here.empty()) launch_tasks(here, /*staged=*/false, /*on_coord=*/b_.await_all || head_next_);
}

void HipComm::launch_update(const UpdateSpec& u) {
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

bool HipComm::fused_ok(const UpdateSpec& u, const std::vector<int64_t>& posted) const {
  const size_t es = u.dtype == MPA_F64 ? 8 : 4;
  if (b_.n > kMaxEpochChunks || int64_t(u.w.size()) != b_.n || b_.rl != size_t(u.elems) * es ||
      b_.sl != size_t(u.elems) * (u.msg_bf16 ? 2 : es) || b_.sendbuf != (u.msg_bf16 ? (const uint8_t*)u.mirror : (const uint8_t*)u.x))
    return false;
  size_t ndst = 0, ndoor = 0;
  for (int64_t rank : posted) {
    const HipWorker& w = w_[size_t(rank - 1)];
    ndst += w.remote ? 2 : 1;
    ndoor += w.remote ? (w.path_dev ? 2 : 1) : 0;
  }
  return ndst <= size_t(kMaxEpochDst) && ndoor <= size_t(kMaxDoorbells);
}

bool HipComm::tail_fits(const std::vector<int64_t>& posted, const UpdateSpec& u) const {
  if (!fused_tail_ || posted.empty() || u.msg_bf16 || u.mirror) return false;
  int cp = -1;
  size_t local = 0, remote = 0;
  for (int64_t rank : posted) {
    const HipWorker& w = w_[size_t(rank - 1)];
    if (w.remote) {  // rank 0: the tail waits for its completion word and rings its doorbells
      ++remote;
      continue;
    }
    const TaskSpec& ts = tasks_[size_t(rank - 1)];
    if (ts.kind != MPA_TASK_LSQ || !ts.delays_ns.empty() || ts.dtype != u.dtype) return false;
    const int c = lsq_cols_pad(ts.dtype, int(ts.cols));
    if (c > kLsqWideSlice) return false;  // wide rows: two launches, no fused tail
    if (cp >= 0 && c != cp) return false;
    cp = c;
    ++local;
  }
  return local >= 1 && local <= size_t(kMaxLsqTasks) && remote <= size_t(kMaxEpochChunks);
}

// The epoch step rides at the head of the task launch (flush) when that launch is the whole
// epoch: every worker of the pool posted by this flush, all local undelayed least-squares
// tasks of one kernel shape, nothing held back.  The launch then runs on the coordinator
// stream, where the epoch kernel would have run.
bool HipComm::head_fits(const std::vector<int64_t>& posted, const UpdateSpec& u) const {
  // the launch is the held re-dispatches (which join it) and this flush's posts
  if (!fused_head_ || int64_t(posted.size() + held_.size()) != b_.n || hold_next_ || u.msg_bf16 || u.mirror)
    return false;
  int cp = -1;
  for (int64_t rank : launch_ranks()) {
    const HipWorker& w = w_[size_t(rank - 1)];
    const TaskSpec& ts = tasks_[size_t(rank - 1)];
    if (w.remote || ts.kind != MPA_TASK_LSQ || !ts.delays_ns.empty() || ts.dtype != u.dtype) return false;
    const int c = lsq_cols_pad(ts.dtype, int(ts.cols));
    if (c > kLsqWideSlice || (cp >= 0 && c != cp)) return false;
    cp = c;
  }
  return !posted.empty() && posted.size() + held_.size() <= size_t(kMaxLsqTasks);
}

// flush_stale() in the descent loop: every re-dispatch of this flush is held, so nothing needs
// to run now -- the pending harvests (the stale reply among them) and the held workers'
// messages go into the next step, ahead of its update, as this flush would have ordered them.
bool HipComm::defer_stale() {
  if (!hold_next_ || !defer_end_ || has_update_ || posts_.empty() || !defer_ok_ ||
      stale_deferred_.size() + posts_.size() > size_t(kMaxEpochDst0))
    return false;
  for (int64_t rank : posts_) {
    const HipWorker& w = w_[size_t(rank - 1)];
    const TaskSpec& ts = tasks_[size_t(rank - 1)];
    if (w.remote || (ts.kind != MPA_TASK_LSQ && ts.kind != MPA_TASK_LSQ_BATCH) || !ts.delays_ns.empty()) return false;
  }
  for (int64_t rank : posts_) stale_deferred_.push_back({b_.sendbuf, const_cast<uint8_t*>(w_[size_t(rank - 1)].x), b_.sl});
  launch_local(posts_);  // every one of them is held (hold_next_)
  n_deferred_ += int64_t(posts_.size());
  posts_.clear();
  return true;
}

void HipComm::run_deferred() {
  if (stale_deferred_.empty()) return;
  cancel_pre();
  ExchangeBuilder xb(ticket_, &ticket_count_, coord_);
  const size_t nb = has_update_ ? harv_before_ : harv_.size();  // harvests due before the update
  for (size_t k = 0; k < nb; ++k) add_harvest(xb, harv_[k]);
  for (const auto& d : stale_deferred_) xb.copy(d.src, d.dst, d.bytes);
  xb.launch();
  harv_.erase(harv_.begin(), harv_.begin() + std::ptrdiff_t(nb));
  if (has_update_) harv_before_ = 0;
  stale_deferred_.clear();
}

void HipComm::emit_epoch(const std::vector<Harvest>& hv, size_t before, const std::vector<int64_t>& posted,
                const UpdateSpec& u, hipStream_t s) {
  EpochArgs a = epoch_args(hv, before, posted, u);
  ++n_epoch_;
  if (a.ndoor > 0) {
    a.ticket = ticket_;
    a.ticket_base = ticket_count_;
    ticket_count_ += uint32_t(epoch_grid(u.dtype, a));
  }
  if (timing_ && x_seq_++ % uint64_t(timing_period_) == 0) {
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

EpochArgs HipComm::epoch_args(const std::vector<Harvest>& hv, size_t before, const std::vector<int64_t>& posted,
                     const UpdateSpec& u) const {
  EpochArgs a;
  std::memset(static_cast<void*>(&a), 0, sizeof a);  // padding too: pre_consume compares bytes
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
  a.sys_fence = msg_wt_ ? 0u : 1u;
  for (const auto& d : stale_deferred_) a.dst0[a.ndst0++] = d.dst;  // (deferred_fit: callers check)
  for (int64_t rank : posted) {
    const HipWorker& w = w_[size_t(rank - 1)];
    a.dst[a.ndst++] = b_.isendbuf + size_t(w.slot) * b_.sl;
    if (w.remote) {
      if (msg_wt_) a.dst_sys |= 1u << a.ndst;  // another process reads it: written through
      a.dst[a.ndst++] = msg_dst(w);
      a.door[a.ndoor] = w.box_door_dev;
      a.doorval[a.ndoor++] = w.seq;
      if (w.path_dev) {  // the device doorbell a device-armed task of the worker waits on
        a.door[a.ndoor] = peer_door(w);
        a.doorval[a.ndoor++] = w.seq;
      }
    }
  }
  return a;
}

void HipComm::maybe_ahead() {
  // an ahead epoch whose step already ran in the previous launch's fused tail must be
  // enqueued now: the descent loop that set it up guarantees it (anything else would apply
  // that update twice)
  auto skip = [this]() {
    if (tail_pending_) fail(MPA_ERROR, "fused tail: the epoch it prepared was not enqueued ahead");
  };
  if (ahead_left_ <= 0 || !b_.await_all || int64_t(call_posts_.size()) != b_.n || !held_.empty()) return skip();
  run_deferred();  // (launch-ahead runs at nwait = n: a held stale re-dispatch is rare there)
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
    if (w.remote && !tail_pending_) {  // (a pending tail waited for them in the previous launch)
      if (g_wait_value_ops) {
        HIPCHECK(hipStreamWaitValue64(coord_, region_->dev(&w.box->done), w.seq, hipStreamWaitValueGte, ~0ull));
      } else {
        if (ww.n == kMaxWaitWords) {
          HIPCHECK(launch_wait_words(ww, coord_));
          ww.n = 0;
        }
        ww.word[ww.n] = remote_done_word(w);
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
    // the tail dispatches the epoch after this one: remote doorbells take its task numbers,
    // and it first waits for this epoch's remote completions
    for (int d = 0; d < tail_args_.ndoor; ++d) tail_args_.doorval[d] += 1;
    tail_ranks_ = 0;
    tail_nwait_ = 0;
    for (int64_t rank : posted) {
      const HipWorker& w = w_[size_t(rank - 1)];
      if (!w.remote) {
        ++tail_ranks_;
        continue;
      }
      tail_word_[tail_nwait_] = remote_done_word(w);
      tail_target_[tail_nwait_++] = w.seq;
    }
    tail_next_ = true;
    tail_pending_ = true;
  }
  launch_local(posted);
  MPA_HSTAMP('A', posted.front(), w_[size_t(posted.front() - 1)].seq);
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

int64_t HipComm::counter(const char* name) const {
  const std::string k = name;
  if (k == "held") return n_held_;
  if (k == "held_joined") return n_held_joined_;
  if (k == "held_alone") return n_held_alone_;
  if (k == "gate_steps") return int64_t(gate_steps_taken());
  if (k == "head_steps") return n_head_;    // epoch steps run at the head of a task launch
  if (k == "epoch_kernels") return n_epoch_;  // epoch steps run as their own epoch kernel
  if (k == "prearmed") return n_prearmed_;   // head steps whose launch was pre-armed
  if (k == "stale_deferred") return n_deferred_;  // held re-dispatches whose messages joined the next step
  if (k == "task_launches") return n_task_launches_.load(std::memory_order_relaxed);  // least-squares launches
  if (k == "prearm_cancelled") return n_pre_cancel_;
  if (k == "prearm_same") return n_pre_same_;  // released with the step's predicted arguments
  if (k == "armed") return n_armed_;  // server: tasks launched device-armed (some may be cancelled)
  if (k == "sleeps") return n_sleeps_;  // delayed tasks queued behind a device deadline (deadline_kernel)
  if (k == "clock_samples") return n_clock_samples_.load(std::memory_order_relaxed);  // host <-> device clock samples behind the deadlines
  if (k == "timer_late") return n_timer_late_.load(std::memory_order_relaxed);  // > 1 ms late timer launches
  if (k == "queues") return queue_streams(dev_);  // CU-masked streams (HSA queues) the process holds
  if (k == "queues_past_cap") return queues_past_cap();
  if (k == "reserved_cus") return reserve_cus_ ? kReservedCus : 0;  // CUs this process's task streams leave out
  if (k == "shared_worker_streams") {  // workers whose stream another worker or comm also uses
    int64_t k2 = 0;
    for (const auto& w : w_)
      if (w.stream && stream_shared(w.stream)) ++k2;
    return k2;
  }
  return -1;
}

void HipComm::watchdog(Clock::time_point t0, bool timeout) {
  check_timer();
  const unsigned e = device_error();
  if (e) fail(MPA_DEVICE_ERROR, "device-side error word 0x%x (an in-kernel wait timed out)", e);
  for (auto& w : w_)
    if (w.stream) check_stream(w.stream);
  for (auto& s : launch_streams_) check_stream(s);
  if (timeout && timeout_s_ > 0 && std::chrono::duration<double>(Clock::now() - t0).count() > timeout_s_)
    fail(MPA_DEVICE_ERROR, "waited more than %.0f s for a worker (MPA_WAIT_TIMEOUT_S)", timeout_s_);
}

void HipComm::check_task(int64_t rank, const TaskSpec& ts, size_t sl, size_t rl) {
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
void hip_set_timing(Comm* c, int period) { static_cast<HipComm*>(c)->set_timing(period); }
void hip_timing(Comm* c, double out[4]) { static_cast<HipComm*>(c)->timing(out); }
void hip_exchange_timing(Comm* c, double out[3]) { static_cast<HipComm*>(c)->exchange_timing(out); }
void hip_set_trace(Comm* c, int64_t capacity) { static_cast<HipComm*>(c)->set_trace(capacity); }
int64_t hip_read_trace(Comm* c, int64_t* out, int64_t capacity) { return static_cast<HipComm*>(c)->read_trace(out, capacity); }

// ---- task trace -------------------------------------------------------------------------
void HipComm::trace_post(HipWorker& w, int64_t rank) {
  w.tslot = -1;
  if (!trace_ || trace_n_ >= trace_cap_) return;
  w.tslot = trace_n_++;
  int64_t* e = trace_ + w.tslot * kTraceFields;
  for (int k = 0; k < kTraceFields; ++k) e[k] = 0;
  e[kTRank] = rank;
  e[kTSeq] = int64_t(w.seq);
  e[kTPost] = int64_t(mono_ns());
}

void HipComm::gate_seen(int64_t rank, uint64_t seq, uint64_t step_begin_ns) {
  const HipWorker& w = w_[size_t(rank - 1)];
  int64_t* e = trace_entry(w);
  if (e && uint64_t(e[kTSeq]) == seq && !e[kTSeen]) {
    e[kTGate] = int64_t(step_begin_ns);
    e[kTSeen] = int64_t(mono_ns());
  }
}

// (device ticks, host ns) of one moment: the tightest of 16 launch -> sync round trips of a
// kernel that stores s_memrealtime, the host time taken as the round trip's midpoint (the
// error is at most half the round trip, ~10 us: the trace is for millisecond-scale splits)
void HipComm::calibrate(int64_t* ticks, int64_t* ns) {
  int64_t best = INT64_MAX;
  for (int k = 0; k < 16; ++k) {
    __atomic_store_n(clock_probe_, 0ull, __ATOMIC_SEQ_CST);
    const int64_t t0 = int64_t(mono_ns());
    HIPCHECK(launch_clock_probe(reinterpret_cast<unsigned long long*>(clock_probe_), coord_));
    for (uint64_t spins = 0; __atomic_load_n(clock_probe_, __ATOMIC_ACQUIRE) == 0; ++spins) {
      if ((spins & 0xFFFF) == 0xFFFF && int64_t(mono_ns()) - t0 > 100000000) {  // 100 ms: a busy stream
        HIPCHECK(hipStreamSynchronize(coord_));
        break;
      }
      __builtin_ia32_pause();
    }
    const int64_t t1 = int64_t(mono_ns());
    if (t1 - t0 < best) {
      best = t1 - t0;
      *ticks = int64_t(__atomic_load_n(clock_probe_, __ATOMIC_ACQUIRE));
      *ns = t0 + (t1 - t0) / 2;
    }
    HIPCHECK(hipStreamSynchronize(coord_));
  }
}

void HipComm::set_trace(int64_t capacity) {
  if (capacity < 0) fail(MPA_ARGUMENT_ERROR, "trace capacity < 0");
  drain_deferred();                  // no timer-deferred launch still holds an entry of the old buffer
  HIPCHECK(hipDeviceSynchronize());  // no task still stamps it
  for (auto& w : w_) w.tslot = -1;
  if (trace_) HIPCHECK(hipHostFree(trace_));
  trace_ = nullptr;
  trace_cap_ = trace_n_ = 0;
  if (capacity == 0) return;
  HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&trace_), size_t(capacity) * kTraceFields * sizeof(int64_t),
                         hipHostMallocCoherent | hipHostMallocMapped));
  if (!clock_probe_)
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&clock_probe_), 64, hipHostMallocCoherent | hipHostMallocMapped));
  trace_cap_ = capacity;
  calibrate(&cal_ticks0_, &cal_ns0_);
}

int64_t HipComm::read_trace(int64_t* out, int64_t capacity) {
  if (!trace_) return 0;
  HIPCHECK(hipDeviceSynchronize());
  int64_t t1 = 0, n1 = 0;
  calibrate(&t1, &n1);
  // device ticks -> host ns through the two calibrations (rate and offset)
  const double rate = t1 > cal_ticks0_ ? double(n1 - cal_ns0_) / double(t1 - cal_ticks0_) : 1e9 / rt_hz_;
  const int64_t n = trace_n_ < capacity ? trace_n_ : capacity;
  for (int64_t j = 0; j < n; ++j) {
    const int64_t* e = trace_ + j * kTraceFields;
    int64_t* o = out + j * kTraceFields;
    for (int k = 0; k < kTraceFields; ++k) o[k] = e[k];
    for (int k : {int(kTStart), int(kTPub)})
      o[k] = e[k] ? cal_ns0_ + int64_t(std::llround(double(e[k] - cal_ticks0_) * rate)) : 0;
  }
  return n;
}
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

void hip_set_defer_end(Comm* c, bool on, bool prearm_ok) { static_cast<HipComm*>(c)->set_defer_end_flush(on, prearm_ok); }
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
