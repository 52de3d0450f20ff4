// SIM transport: a deterministic virtual-clock communicator whose workers run the
// reference's test worker programs (echo, test/kmap1.jl:23-33, test/kmap2.jl:76-99) on
// host buffers.  It exists to test the pool state machine on machines without a GPU; it
// is never selected implicitly and carries no least-squares compute.
//
// It defers copies exactly like the HIP transport (the sendbuf -> isendbuf slot copy and
// the irecvbuf -> recvbuf harvest copies happen at flush()/end_call()), so a missing
// flush in the state machine shows up as wrong recvbuf bytes in the CPU tests.
#include <cstring>

#include "comm.hpp"

namespace mpa {
namespace {

struct SimWorker {
  int64_t t = 0;          // messages served (kmap2.jl:82-84)
  int64_t done_ns = 0;    // completion time of the outstanding task
  int64_t slot = -1;      // pool position of the outstanding request
  bool started = false;   // its send has been flushed
  bool delivered = true;  // reply written into irecv chunk
  uint8_t* irecv = nullptr;
  const uint8_t* isend = nullptr;
  size_t sl = 0, rl = 0;
};

class SimComm final : public Comm {
 public:
  explicit SimComm(int64_t n) : Comm(n), w_(size_t(n)) {}
  int transport() const override { return MPA_TRANSPORT_SIM; }

  void begin_call(const CallBufs& b) override { b_ = b; }

  void post(int64_t i, int64_t rank, int64_t tag) override {
    (void)tag;
    if (shutdown_) fail(MPA_ERROR, "comm has been shut down");
    SimWorker& w = w_[size_t(rank - 1)];
    w.slot = i;
    w.started = false;
    w.delivered = false;
    w.isend = b_.isendbuf + size_t(i) * b_.sl;
    w.irecv = b_.irecvbuf + size_t(i) * b_.rl;
    w.sl = b_.sl;
    w.rl = b_.rl;
    pending_posts_.push_back(rank);
  }

  void harvest(int64_t i, int64_t rank) override {
    (void)rank;
    pending_harvest_.push_back(i);
  }

  bool test(int64_t i, int64_t rank) override {
    (void)i;
    SimWorker& w = w_[size_t(rank - 1)];
    if (!w.started || w.done_ns > now_) return false;
    deliver(rank);
    return true;
  }

  int64_t waitany(int64_t n, const int64_t* ranks, const uint8_t* live) override {
    int64_t best = -1;
    for (int64_t i = 0; i < n; ++i) {
      if (!live[i]) continue;
      const SimWorker& w = w_[size_t(ranks[i] - 1)];
      if (w.done_ns <= now_) { deliver(ranks[i]); return i; }
      if (best < 0 || w.done_ns < w_[size_t(ranks[best] - 1)].done_ns) best = i;
    }
    if (best < 0) return -1;
    now_ = w_[size_t(ranks[best] - 1)].done_ns;
    deliver(ranks[best]);
    return best;
  }

  void waitall(int64_t n, const int64_t* ranks, const uint8_t* live) override {
    for (int64_t i = 0; i < n; ++i)
      if (live[i] && w_[size_t(ranks[i] - 1)].done_ns > now_) now_ = w_[size_t(ranks[i] - 1)].done_ns;
    for (int64_t i = 0; i < n; ++i)
      if (live[i]) deliver(ranks[i]);
  }

  void flush() override {
    for (int64_t i : pending_harvest_)
      std::memcpy(b_.recvbuf + size_t(i) * b_.rl, b_.irecvbuf + size_t(i) * b_.rl, b_.rl);
    pending_harvest_.clear();
    for (int64_t rank : pending_posts_) {
      SimWorker& w = w_[size_t(rank - 1)];
      std::memcpy(const_cast<uint8_t*>(w.isend), b_.sendbuf, b_.sl);
      w.t += 1;
      const TaskSpec& ts = tasks_[size_t(rank - 1)];
      int64_t d = compute_ns_;
      if (!ts.delays_ns.empty()) d += ts.delays_ns[size_t((w.t - 1) % int64_t(ts.delays_ns.size()))];
      w.done_ns = now_ + d;
      w.started = true;
    }
    pending_posts_.clear();
  }

  void end_call() override { flush(); }
  uint64_t now_ns() override { return uint64_t(now_); }

  int64_t tasks_done(int64_t rank) override {
    const SimWorker& w = w_[size_t(rank - 1)];
    return w.delivered ? w.t : w.t - 1;
  }
  void shutdown() override { shutdown_ = true; }

  void set_compute(int64_t ns) { compute_ns_ = ns; }
  void advance(int64_t dt) { now_ += dt; }
  int64_t now() const { return now_; }

 private:
  void deliver(int64_t rank) {
    SimWorker& w = w_[size_t(rank - 1)];
    if (w.delivered) return;
    w.delivered = true;
    const int kind = tasks_[size_t(rank - 1)].kind;
    std::memset(w.irecv, 0, w.rl);
    if (kind == MPA_TASK_KMAP1) {
      const double v = double(rank);
      std::memcpy(w.irecv, &v, w.rl < 8 ? w.rl : 8);
    } else if (kind == MPA_TASK_KMAP2) {
      double v[3] = {double(rank), double(w.t), 0.0};
      std::memcpy(&v[2], w.isend, w.sl < 8 ? w.sl : 8);
      std::memcpy(w.irecv, v, w.rl < sizeof v ? w.rl : sizeof v);
    } else {  // ECHO (the default worker program)
      std::memcpy(w.irecv, w.isend, w.sl < w.rl ? w.sl : w.rl);
    }
  }

  std::vector<SimWorker> w_;
  std::vector<int64_t> pending_posts_, pending_harvest_;
  CallBufs b_;
  int64_t now_ = 0, compute_ns_ = 0;
};

}  // namespace

Comm* make_sim_comm(int64_t nworkers) { return new SimComm(nworkers); }
void sim_set_compute(Comm* c, int64_t ns) { static_cast<SimComm*>(c)->set_compute(ns); }
void sim_advance(Comm* c, int64_t dt) { static_cast<SimComm*>(c)->advance(dt); }
int64_t sim_now(const Comm* c) { return static_cast<const SimComm*>(c)->now(); }

}  // namespace mpa
