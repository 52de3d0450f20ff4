// HOST transport: the multi-process mailbox protocol of the HIP transport (shm.hpp,
// transport_hip.cpp roles COORD / SERVER) with host-memory buffers and host-executed
// worker programs (echo, test/kmap1.jl, test/kmap2.jl).  It exists so that the N > 1
// control plane (shared-memory mailboxes, doorbells, completion words, pause / shutdown,
// one process per rank) is tested on machines without a GPU; it carries no least-squares
// compute and is never selected implicitly.
//
// Same ordering as the device path: a flush copies harvested replies out first, then
// writes messages and rings doorbells (release); a server publishes a reply's bytes before
// its completion word (release); the coordinator acquires the completion word before
// copying the reply.  Injected delays are honoured by the server: a task completes at
// (doorbell seen) + delay.
#include <chrono>
#include <cstring>
#include <memory>
#include <thread>

#include "comm.hpp"
#include "shm.hpp"

namespace mpa {
namespace {

using Clock = std::chrono::steady_clock;

int64_t now_ns_host() {
  return int64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count());
}

// reply of the reference's test worker programs
void run_worker_program(int kind, int64_t rank, uint64_t t, const uint8_t* msg, size_t sl, uint8_t* out, size_t rl) {
  std::memset(out, 0, rl);
  if (kind == MPA_TASK_KMAP1) {
    const double v = double(rank);
    std::memcpy(out, &v, rl < 8 ? rl : 8);
  } else if (kind == MPA_TASK_KMAP2) {
    double v[3] = {double(rank), double(t), 0.0};
    std::memcpy(&v[2], msg, sl < 8 ? sl : 8);
    std::memcpy(out, v, rl < sizeof v ? rl : sizeof v);
  } else {
    std::memcpy(out, msg, sl < rl ? sl : rl);
  }
}

struct HostWorker {
  bool here = false, remote = false;
  unsigned long long seq = 0;
  BoxHeader* box = nullptr;
  int64_t slot = -1;
  // server: a task seen but not yet published
  bool pending = false;
  int64_t due_ns = 0;
  unsigned long long local_done = 0;  // coordinator-local workers
};

class HostDistComm final : public Comm {
 public:
  HostDistComm(int64_t n, const int* placement, int my_rank, ShmRegion* region)
      : Comm(n), w_(size_t(n)), region_(region), my_rank_(my_rank) {
    for (int64_t i = 0; i < n; ++i) {
      HostWorker& w = w_[size_t(i)];
      w.here = placement[i] == my_rank;
      w.remote = my_rank == 0 && !w.here;
      w.box = region_->box(i + 1);
    }
  }
  ~HostDistComm() override { delete region_; }

  int transport() const override { return MPA_TRANSPORT_HOST; }

  void begin_call(const CallBufs& b) override {
    if (my_rank_ != 0) fail(MPA_ERROR, "asyncmap!/waitall! run on rank 0; this process serves workers (mpa_comm_serve)");
    b_ = b;
  }

  void post(int64_t i, int64_t rank, int64_t tag) override {
    (void)tag;
    if (shutdown_) fail(MPA_ERROR, "comm has been shut down");
    HostWorker& w = w_[size_t(rank - 1)];
    if (w.remote && (b_.sl > region_->max_msg() || b_.rl > region_->max_msg()))
      fail(MPA_DIMENSION_MISMATCH, "messages of %zu / %zu bytes exceed the communicator's mailbox of %zu bytes", b_.sl,
           b_.rl, region_->max_msg());
    if (!w.remote && tasks_[size_t(rank - 1)].kind == MPA_TASK_NONE)
      fail(MPA_ERROR, "worker %lld has no task registered (mpa_comm_set_task_*)", (long long)rank);
    w.slot = i;
    w.seq += 1;
    posts_.push_back(rank);
  }

  void harvest(int64_t i, int64_t rank) override { harv_.push_back({i, rank}); }

  bool test(int64_t i, int64_t rank) override {
    (void)i;
    return done(rank);
  }

  int64_t waitany(int64_t n, const int64_t* ranks, const uint8_t* live) override {
    bool any = false;
    for (int64_t i = 0; i < n; ++i) any |= live[i] != 0;
    if (!any) return -1;
    for (;;) {
      for (int64_t i = 0; i < n; ++i)
        if (live[i] && done(ranks[i])) return i;
      std::this_thread::yield();
    }
  }

  void waitall(int64_t n, const int64_t* ranks, const uint8_t* live) override {
    for (int64_t i = 0; i < n; ++i)
      while (live[i] && !done(ranks[i])) std::this_thread::yield();
  }

  void flush() override {
    for (const auto& h : harv_) {
      const HostWorker& w = w_[size_t(h.rank - 1)];
      const uint8_t* src = w.remote ? region_->reply(h.rank) : b_.irecvbuf + size_t(h.slot) * b_.rl;
      std::memcpy(b_.recvbuf + size_t(h.slot) * b_.rl, src, b_.rl);
    }
    harv_.clear();
    for (int64_t rank : posts_) {
      HostWorker& w = w_[size_t(rank - 1)];
      uint8_t* slot = b_.isendbuf + size_t(w.slot) * b_.sl;
      std::memcpy(slot, b_.sendbuf, b_.sl);
      if (w.remote) {
        std::memcpy(region_->msg(rank), b_.sendbuf, b_.sl);
        w.box->msg_bytes = b_.sl;
        w.box->reply_bytes = b_.rl;
        __atomic_store_n(&w.box->doorbell, w.seq, __ATOMIC_RELEASE);
      } else {  // a worker of rank 0 itself: runs now
        run_worker_program(tasks_[size_t(rank - 1)].kind, rank, w.seq, slot, b_.sl,
                           b_.irecvbuf + size_t(w.slot) * b_.rl, b_.rl);
        __atomic_store_n(&w.local_done, w.seq, __ATOMIC_RELEASE);
      }
    }
    posts_.clear();
  }

  void end_call() override { flush(); }
  uint64_t now_ns() override { return uint64_t(now_ns_host()); }

  int64_t tasks_done(int64_t rank) override { return int64_t(done_word(rank)); }

  void shutdown() override {
    gate_off();
    if (my_rank_ == 0) {
      for (int64_t r = 1; r <= nworkers_; ++r)
        while (!done(r)) std::this_thread::yield();
      __atomic_store_n(&region_->header()->shutdown, 1ull, __ATOMIC_RELEASE);
    }
    shutdown_ = true;
  }

  void serve() {
    if (my_rank_ == 0) fail(MPA_ERROR, "mpa_comm_serve is for worker processes (rank != 0)");
    ShmHeader* h = region_->header();
    const uint64_t gen0 = __atomic_load_n(&h->gen, __ATOMIC_ACQUIRE);
    for (;;) {
      const bool stop =
          __atomic_load_n(&h->shutdown, __ATOMIC_ACQUIRE) || __atomic_load_n(&h->gen, __ATOMIC_ACQUIRE) != gen0;
      const int64_t now = now_ns_host();
      bool busy = false;
      for (int64_t r = 1; r <= nworkers_; ++r) {
        HostWorker& w = w_[size_t(r - 1)];
        if (!w.here) continue;
        if (!w.pending && !stop) {
          const unsigned long long db = __atomic_load_n(&w.box->doorbell, __ATOMIC_ACQUIRE);
          if (db != w.seq) {
            if (db != w.seq + 1) fail(MPA_ERROR, "mailbox protocol: worker %lld doorbell %llu after %llu", (long long)r, db, w.seq);
            w.seq = db;
            const TaskSpec& ts = tasks_[size_t(r - 1)];
            if (ts.kind == MPA_TASK_NONE) fail(MPA_ERROR, "worker %lld has no task registered", (long long)r);
            int64_t d = 0;
            if (!ts.delays_ns.empty()) d = ts.delays_ns[size_t((int64_t(w.seq) - 1) % int64_t(ts.delays_ns.size()))];
            w.pending = true;
            w.due_ns = now + d;
          }
        }
        if (w.pending) {
          busy = true;
          if (now >= w.due_ns) {
            const TaskSpec& ts = tasks_[size_t(r - 1)];
            run_worker_program(ts.kind, r, w.seq, region_->msg(r), size_t(w.box->msg_bytes), region_->reply(r),
                               size_t(w.box->reply_bytes));
            __atomic_store_n(&w.box->done, w.seq, __ATOMIC_RELEASE);
            w.pending = false;
          }
        }
      }
      if (stop && !busy) break;
      std::this_thread::yield();
    }
  }

  void pause_servers() {
    if (my_rank_ != 0) fail(MPA_ERROR, "only rank 0 pauses the servers");
    __atomic_fetch_add(&region_->header()->gen, 1ull, __ATOMIC_RELEASE);
  }

 private:
  struct Harvest {
    int64_t slot, rank;
  };
  unsigned long long done_word(int64_t rank) const {
    const HostWorker& w = w_[size_t(rank - 1)];
    return w.remote || my_rank_ != 0 ? __atomic_load_n(&w.box->done, __ATOMIC_ACQUIRE)
                                     : __atomic_load_n(&w.local_done, __ATOMIC_ACQUIRE);
  }
  bool done(int64_t rank) const {
    const unsigned long long seq = w_[size_t(rank - 1)].seq;
    return done_word(rank) >= seq && gate_open(rank, seq);
  }

  // gated replay hooks (gate.cpp)
  bool gate_supported() const override { return my_rank_ == 0; }
  uint64_t gate_posted(int64_t rank) override { return w_[size_t(rank - 1)].seq; }
  uint64_t gate_finished(int64_t rank) override { return done_word(rank); }
  void gate_poll(double waited_s) override {
    if (waited_s > 600) fail(MPA_ERROR, "gated replay: waited more than 600 s for a released task");
  }

  std::vector<HostWorker> w_;
  ShmRegion* region_;
  int my_rank_;
  std::vector<int64_t> posts_;
  std::vector<Harvest> harv_;
  CallBufs b_;
};

}  // namespace

Comm* make_host_dist_comm(int64_t nworkers, const int* placement, int my_rank, const char* shm_name, size_t max_msg) {
  if (!placement) fail(MPA_ARGUMENT_ERROR, "placement is NULL");
  if (!shm_name || !*shm_name) fail(MPA_ARGUMENT_ERROR, "shared memory name is empty");
  std::unique_ptr<ShmRegion> r(my_rank == 0 ? ShmRegion::create(shm_name, nworkers, max_msg, false)
                                            : ShmRegion::attach(shm_name, false));
  if (r->nworkers() != nworkers) fail(MPA_ARGUMENT_ERROR, "shared memory holds %lld workers, comm has %lld",
                                      (long long)r->nworkers(), (long long)nworkers);
  Comm* c = new HostDistComm(nworkers, placement, my_rank, r.get());
  r.release();
  return c;
}
void host_serve(Comm* c) { static_cast<HostDistComm*>(c)->serve(); }
void host_pause_servers(Comm* c) { static_cast<HostDistComm*>(c)->pause_servers(); }

}  // namespace mpa
