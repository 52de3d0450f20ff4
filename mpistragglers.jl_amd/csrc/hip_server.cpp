// HipComm, worker processes (N > 1): the doorbell loop of mpa_comm_serve (the
// reference's worker_main, examples/iterative_example.jl:55-82), pre-armed tasks and their
// cancellation, the HIP IPC device-memory payload path over xGMI and the host-mailbox fallback.
#include "hip_transport.hpp"

namespace mpa {

void HipComm::serve() {
  if (role_ != SERVER) fail(MPA_ERROR, "mpa_comm_serve is for worker processes (rank != 0)");
  ShmHeader* h = region_->header();
  const uint64_t gen0 = __atomic_load_n(&h->gen, __ATOMIC_ACQUIRE);
  const auto t0 = Clock::now();
  struct Disarm {
    HipComm* c;
    ~Disarm() { c->disarm_all(); }
  } disarm_guard{this};
  std::vector<int64_t> fresh;
  // the doorbell poll between tasks: hot for 5 ms after the last task (an epoch's gap between a
  // worker's reply and its next doorbell), then yielding; with a 50 us window the serve loops of
  // the one-GPU eight-process tests yielded their cores between epochs and saw doorbells
  // milliseconds late on a loaded box (r06h)
  PoliteSpin idle;
  idle.yield_cold = true;
  idle.hot_ns = kServerHotSpinNs;
  for (int64_t r = 1; r <= nworkers_; ++r)
    if (w_[size_t(r - 1)].here && server_path(r) && armable(r)) arm_up(r);
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
          if (armable(r)) arm_up(r);
        }
        continue;
      }
      if (w.armed) {
        // the oldest armed task ran: check what rank 0 posted against what it was armed for,
        // then queue the next one behind the youngest
        const unsigned long long oldest = w.seq - unsigned(w.armed) + 1;
        if (__atomic_load_n(w.flag_host, __ATOMIC_ACQUIRE) < oldest) continue;
        w.armed -= 1;
        MPA_HSTAMP('D', r, oldest);
        check_task(r, tasks_[size_t(r - 1)], size_t(w.box->msg_bytes), size_t(w.box->reply_bytes));
        progress = true;
        if (armable(r)) arm_up(r);
        continue;
      }
      const unsigned long long db = __atomic_load_n(&w.box->doorbell, __ATOMIC_ACQUIRE);
      if (db == w.seq) continue;
      MPA_HSTAMP('B', r, db);
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
            if (!w.here || !w.path_known || w.armed > 0 || std::find(fresh.begin(), fresh.end(), r) != fresh.end()) continue;
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
            postable += w.here && w.path_known && w.armed == 0 &&
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
      MPA_HSTAMP('T', fresh.front(), w_[size_t(fresh.front() - 1)].seq);
      idle = PoliteSpin{};
      idle.yield_cold = true;
      idle.hot_ns = kServerHotSpinNs;
    } else if (!progress) {
      if ((spins & 0xFFF) == 0xFFF) watchdog(t0, /*timeout=*/false);
      idle();
    } else {
      idle = PoliteSpin{};  // busy again: the next idle stretch starts hot
      idle.yield_cold = true;
      idle.hot_ns = kServerHotSpinNs;
    }
  }
}

// Device-armed tasks: least-squares workers whose messages arrive in this GPU's
// slot (device payload path).  MPA_ARM: 0 never, 1 every such worker, 2 (default) where the
// process serves one worker (the N = 8 placement; a process with several workers launches the
// tasks of a flush as one batch instead).  The in-kernel wait (MPA_ARM_WAIT=kernel: every
// workgroup of the armed launch waits) is refused by the default on a GPU that rank 0 also uses:
// the waiting grids held the CUs rank 0's kernels needed to ring them
// (profiles/r03_rehearsal_n248.txt); the default one-wave wait (door_wait_kernel)
// holds nothing anyone needs.  A worker with injected delays is armed too (round 6), behind the
// one-wave wait, which sleeps its delay from the ring on the device: host-launched, its delay
// began only when this process's serve loop saw the doorbell -- milliseconds late on a loaded
// box, when a yielding poll lost its core (the one-GPU k-of-n process tests, r06h).
bool HipComm::armable(int64_t rank) const {
  const TaskSpec& ts = tasks_[size_t(rank - 1)];
  const HipWorker& w = w_[size_t(rank - 1)];
  if (arm_mode_ == 0 || !w.path_dev || !(ts.kind == MPA_TASK_LSQ || ts.kind == MPA_TASK_LSQ_BATCH) ||
      (!ts.delays_ns.empty() && (!arm_wave_ || delay_mode_ == 1)))
    return false;
  if (arm_mode_ == 1) return true;
  int here = 0;
  for (const auto& v : w_) here += v.here;
  if (here != 1) return false;
  return arm_wave_ || w.box->coord_dev != dev_ || arm_force_;
}

// The worker's next task is launched before rank 0 posts it and waits for the worker's device
// doorbell, which rank 0's exchange / epoch kernel stores over xGMI right after the message, so
// ring -> start is a poll of this GPU's memory instead of the serve loop's host poll and a
// launch (19 us of the traced c2 N = 2 epoch).  Default: a one-wave door_wait_kernel with the
// task queued behind it; MPA_ARM_WAIT=kernel: the task kernel's own in-kernel wait (wait_door,
// every workgroup).  Either way the task reads its go word (a cancel) before it replies.
void HipComm::arm(int64_t rank) {
  HipWorker& w = w_[size_t(rank - 1)];
  const TaskSpec& ts = tasks_[size_t(rank - 1)];
  const unsigned long long s = w.seq + 1;
  const int par = int(s & 1);
  w.arm_sbase[par] = w.lsqb_sbase;
  w.arm_tbase[par] = w.lsqb_tbase;
  w.arm_fsbase[par] = w.lsqf_sbase;
  w.arm_ftbase[par] = w.lsqf_tbase;
  w.seq = s;
  unsigned long long* cancel = w.cancel_dev + par;
  w.sl = task_msg_bytes(ts);
  w.rl = w.sl * (ts.kind == MPA_TASK_LSQ_BATCH ? 2 : 1);
  w.x = w.xslot;
  w.out = reply_dst(w);
  hipStream_t st = worker_stream(w);
  unsigned long long* door = arm_wave_ ? nullptr : own_door(w);
  // the injected delay of task s (launch_tasks' schedule index), less the overhead that follows
  // the wait: the task's dispatch behind it, the task, its completion word
  const int64_t delay = ts.delays_ns.empty() ? 0 : ts.delays_ns[size_t((int64_t(s) - 1) % int64_t(ts.delays_ns.size()))];
  const int64_t sleep_ns = delay - deadline_lead_ns_;
  const unsigned long long sleep_ticks = sleep_ns > 0 ? (unsigned long long)(double(sleep_ns) * rt_hz_ / 1e9) : 0ull;
  if (sleep_ticks) n_sleeps_ += 1;
  if (arm_wave_) HIPCHECK(launch_door_wait(own_door(w), s, spin_ticks(), err_dev_, cancel, sleep_ticks, st));
  MPA_HSTAMP('W', rank, s);
  double bytes = 0;
  if (ts.kind == MPA_TASK_LSQ) {
    LsqBatch b = build_lsq_batch({rank}, ts.dtype, &bytes, armed_share());
    b.t[0].go = cancel;
    b.t[0].door = door;
    enqueue_lsq(b, ts.dtype, int(ts.cols), st, bytes, rank);
  } else {
    LsqbLaunch b = build_lsqb_batch({rank}, &bytes, armed_share());
    b.set_go(cancel);
    b.set_door(door);
    enqueue_lsqb(b, st, bytes, rank);
  }
  w.armed += 1;
  n_armed_ += 1;
  MPA_HSTAMP('L', rank, s);
}

void HipComm::disarm_all() {
  if (role_ != SERVER) return;
  for (int64_t r = 1; r <= nworkers_; ++r) {
    HipWorker& w = w_[size_t(r - 1)];
    if (!w.here || !w.armed) continue;
    // release the waiting tasks rank 0 has not rung with the cancel bit (its kernel stores the
    // device word after the shm one): cancel words first, so every workgroup of a released task
    // finds its own; a cancelled task runs but neither writes nor publishes.  Rank 0 has
    // harvested everything it rang before it pauses, so the device word holds the shm value.
    const unsigned long long newest = w.seq, oldest = w.seq - unsigned(w.armed) + 1;
    const unsigned long long rung = __atomic_load_n(&w.box->doorbell, __ATOMIC_ACQUIRE);
    const unsigned long long first = std::max(oldest, rung + 1);  // the first task not rung
    bool cancelled = false;
    if (first <= newest) {
      for (unsigned long long s = first; s <= newest; ++s) __atomic_store_n(w.cancel_host + (s & 1), s, __ATOMIC_SEQ_CST);
      cancelled = door_cas(w, first - 1, newest | kCancelBit);
    }
    (void)hipStreamSynchronize(w.stream);
    if (cancelled) (void)door_cas(w, newest | kCancelBit, first - 1);  // back to "not rung"
    __atomic_store_n(w.cancel_host, 0ull, __ATOMIC_SEQ_CST);
    __atomic_store_n(w.cancel_host + 1, 0ull, __ATOMIC_SEQ_CST);
    // the tasks that did not run: the next serve() session arms them again from the counter
    // bases the first of them started from
    const unsigned long long ran = __atomic_load_n(w.flag_host, __ATOMIC_ACQUIRE);
    if (ran < newest) {
      const int par = int((ran + 1) & 1);
      w.lsqb_sbase = w.arm_sbase[par];
      w.lsqb_tbase = w.arm_tbase[par];
      w.lsqf_sbase = w.arm_fsbase[par];
      w.lsqf_tbase = w.arm_ftbase[par];
      for (unsigned long long s = ran + 1; s <= newest; ++s) void_timing(r);
      w.seq = ran;
    }
    w.armed = 0;
  }
}

int HipComm::arm_depth(int64_t rank) const {
  if (arm_depth_env_) return arm_depth_env_;
  return w_[size_t(rank - 1)].box->coord_dev != dev_ ? 2 : 1;
}

void HipComm::arm_up(int64_t rank) {
  const int d = arm_depth(rank);
  while (w_[size_t(rank - 1)].armed < d) arm(rank);
}

// the worker's device doorbell := desired if it holds expect (a kernel on a launch stream:
// the word is this GPU's fine-grained memory, which rank 0 stores over xGMI); true if it did
bool HipComm::door_cas(const HipWorker& w, unsigned long long expect, unsigned long long desired) {
  hipStream_t s = launch_stream(0);
  unsigned long long* scratch = &cancel_[2 * nworkers_];
  __atomic_store_n(scratch, ~0ull, __ATOMIC_SEQ_CST);  // the word's old value
  HIPCHECK(launch_door_cas(own_door(w), expect, desired, scratch, s));
  HIPCHECK(hipStreamSynchronize(s));
  return __atomic_load_n(scratch, __ATOMIC_ACQUIRE) == expect;
}

void* HipComm::ipc_alloc(size_t bytes, char* handle, volatile uint32_t* state) {
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

void* HipComm::ipc_open(const char* handle, int peer_dev) {
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

void HipComm::decide_path(int64_t rank) {
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

bool HipComm::server_path(int64_t rank) {
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

void HipComm::stage_in(const std::vector<int64_t>& ranks, hipStream_t s) {
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

}  // namespace mpa
