// Transport-facing interface of a communicator (the `comm::MPI.Comm` argument of
// asyncmap!, src/MPIAsyncPools.jl:68) and the worker tasks registered on it.
//
// The pool state machine (pool.cpp) drives a Comm through the MPI point-to-point verbs
// the reference uses: Isend+Irecv! (:137-138, :182-183) -> post(), Test! (:99) -> test(),
// Waitany! (:161) -> waitany(), Waitall! (:212) -> waitall(), and the byte copy
// `recvbufs[i] .= irecvbufs[i]` (:108, :167, :216) -> harvest().  A transport may defer
// harvest copies and posts until flush(); the pool calls flush() wherever the reference's
// program order makes a deferred copy observable (before a worker's irecv chunk can be
// overwritten) and end_call() before returning to the caller.
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <thread>
#include <chrono>
#include <vector>

#include "common.hpp"

namespace mpa {

// A polite poll for the transport's long waits: pause for the first kHotSpinNs of a wait (c1's
// epochs wait microseconds: no system call on that path), then yield the core on every poll --
// while a straggler timer of this process has a launch pending.  The coordinator's wait and the
// timer's final spin are two busy threads of one process; on a core they share, a bare pause loop
// keeps the other one off until the scheduler's time slice ends.  With no timer work (delays as
// device deadlines, or none) the wait keeps pausing: on a loaded box (loadavg 20+) a yield gave
// the core away for a slice and the gated kmap2_n9 replay harvested 1.0-1.4 ms late (r06d, r06e).
// A worker process's idle doorbell poll always yields once cold (yield_cold).  (Sleeping between
// polls instead -- 20 us asked, ~60 us of timer slack got -- moved the gated replays' median
// harvest from 4 to 42 us and their worst from 1.0 to 1.5 ms: r05o.)
constexpr int64_t kHotSpinNs = 50000;
constexpr int64_t kServerHotSpinNs = 5000000;
extern std::atomic<int64_t> g_timer_pending;  // host-timer launches pending in this process
struct PoliteSpin {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  uint32_t n = 0;
  bool cold = false;
  bool yield_cold = false;  // yield once cold whether or not a timer is pending
  int64_t hot_ns = kHotSpinNs;
  void operator()() {
    if (cold && (yield_cold || g_timer_pending.load(std::memory_order_relaxed) > 0)) {
      std::this_thread::yield();
      return;
    }
    __builtin_ia32_pause();
    if ((++n & 63) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::nanoseconds(hot_ns)) cold = true;
  }
};


struct CallBufs {
  const uint8_t* sendbuf = nullptr;
  size_t sl = 0;  // bytes per send slot (sizeof(sendbuf), :80)
  uint8_t* recvbuf = nullptr;
  uint8_t* isendbuf = nullptr;
  uint8_t* irecvbuf = nullptr;
  size_t rl = 0;  // bytes per recv chunk (:81)
  int64_t n = 0;  // pool size
  // the call returns only once every task it posts has completed (integer nwait == n), so
  // a transport may order those tasks on the coordinator's own stream
  bool await_all = false;
};

struct TaskSpec {
  int kind = MPA_TASK_NONE;
  int dtype = MPA_F32;
  int64_t rows = 0, cols = 0, lda = 0;
  int64_t k = 1;  // iterates per message (MPA_TASK_LSQ_BATCH: kLsqbIterates)
  const void* A = nullptr;
  const void* b = nullptr;  // b (rows) or B (rows x k)
  std::vector<int64_t> delays_ns;
};

class Comm {
 public:
  explicit Comm(int64_t nworkers) : nworkers_(nworkers), tasks_(size_t(nworkers)) {}
  virtual ~Comm() = default;
  virtual int transport() const = 0;
  int64_t nworkers() const { return nworkers_; }

  // ---- per-call protocol (pool.cpp) ----
  virtual void begin_call(const CallBufs& b) = 0;
  virtual void post(int64_t i, int64_t rank, int64_t tag) = 0;
  virtual void harvest(int64_t i, int64_t rank) = 0;
  virtual bool test(int64_t i, int64_t rank) = 0;
  virtual int64_t waitany(int64_t n, const int64_t* ranks, const uint8_t* live) = 0;
  virtual void waitall(int64_t n, const int64_t* ranks, const uint8_t* live) = 0;
  virtual void flush() = 0;
  // the flush of a stale worker's re-dispatch inside the wait loop (src/MPIAsyncPools.jl:
  // 177-184); a transport may hold the task's launch back until its next flush or until a
  // wait would block (HIP: the task then joins the next epoch's batched launch)
  virtual void flush_stale() { flush(); }
  // before each waitany of the wait loop: true when the results still owed by tasks posted
  // in phase 2 of this call already satisfy an integer nwait, so a held re-dispatch need not
  // be launched for the call to finish (false: a wait that would block launches it first)
  virtual void set_wait_hold(bool may_hold) { (void)may_hold; }
  virtual void end_call() = 0;
  virtual uint64_t now_ns() = 0;

  // ---- worker registration ----
  TaskSpec& task(int64_t rank) {
    if (rank < 1 || rank > nworkers_) fail(MPA_ARGUMENT_ERROR, "rank %lld is not a worker rank of this comm (1:%lld)",
                                           (long long)rank, (long long)nworkers_);
    return tasks_[size_t(rank - 1)];
  }
  virtual void on_task_changed(int64_t rank) { (void)rank; }
  virtual void on_delays_changed(int64_t rank) { (void)rank; }
  virtual int64_t tasks_done(int64_t rank) = 0;
  virtual void shutdown() = 0;
  bool is_shutdown() const { return shutdown_; }

  // ---- gated replay (mpa_comm_set_gate, gate.cpp) ----
  // A test mode that fixes the completion order to a schedule.  The state machine calls
  // gate() at each of its observation points (pool.cpp: before phase 1 of asyncmap!,
  // before each Waitany! with a live request, before Waitall!); step k of the schedule
  // names the workers that release one more completion there.  A worker's request then
  // reads as complete only once its task has finished AND been released, and gate() waits
  // until every task it releases has finished, so each Test!/Waitany! sees exactly the set
  // of completions the schedule says (the oracle's virtual-clock set, ties included).
  // After the last step the next observation switches the gate off.
  void set_gate(const int* kinds, const int64_t* offsets, const int64_t* ranks, int64_t nsteps);
  void gate(int kind);
  bool gated() const { return gate_on_; }
  size_t gate_steps_taken() const { return gate_step_; }

  // event counters of the transport for tests and diagnostics (mpa_comm_counter); -1 for a
  // name the transport does not count
  virtual int64_t counter(const char* name) const { (void)name; return -1; }

 protected:
  bool gate_open(int64_t rank, uint64_t seq) const { return !gate_on_ || gate_rel_[size_t(rank - 1)] >= seq; }
  void gate_off() { gate_on_ = false; }
  // transport hooks of the gate: tasks posted to / finished by a worker, make sure a posted
  // task is launched (the HIP transport's held re-dispatches), check errors while waiting
  virtual bool gate_supported() const { return false; }
  virtual uint64_t gate_posted(int64_t rank) { (void)rank; return 0; }
  virtual uint64_t gate_finished(int64_t rank) { (void)rank; return 0; }
  virtual void gate_launch(int64_t rank) { (void)rank; }
  virtual void gate_poll(double waited_s) { (void)waited_s; }
  // the gate step that began at step_begin_ns (steady clock) saw task `seq` of `rank` complete
  // (task trace, HipComm)
  virtual void gate_seen(int64_t rank, uint64_t seq, uint64_t step_begin_ns) {
    (void)rank;
    (void)seq;
    (void)step_begin_ns;
  }

  int64_t nworkers_;
  std::vector<TaskSpec> tasks_;
  bool shutdown_ = false;

 private:
  bool gate_on_ = false;
  size_t gate_step_ = 0;
  std::vector<int> gate_kinds_;
  std::vector<int64_t> gate_off_, gate_ranks_;
  std::vector<uint64_t> gate_rel_;  // completions released per worker
};

Comm* make_sim_comm(int64_t nworkers);
// wraps a transport built outside this library (libmpiasyncpools_mpi.so) in a C-ABI handle
::mpa_comm* adopt_comm(Comm* c);
Comm* make_hip_comm(int64_t nworkers, const int* devices);

}  // namespace mpa
