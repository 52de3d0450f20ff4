// MPI transport: the pool over a real MPI communicator whose ranks 1..size-1 run ARBITRARY
// worker programs, as the reference's own examples and tests do
// (examples/iterative_example.jl:55-82, test/kmap1.jl:23-33, test/kmap2.jl:76-99).  It is
// the reference's transport verbatim: post = Isend of the worker's isendbuf slot then Irecv!
// into its irecvbuf chunk (src/MPIAsyncPools.jl:130-138, :178-183), test = Test! (:99),
// waitany = Waitany! (:161), waitall = Waitall! (:212), harvest = the byte copy plus Wait!
// on the send request (:108-113, :167-171, :216-218).  Host buffers; no device work.
//
// Built into its own library (libmpiasyncpools_mpi.so, Makefile target `mpi`) only where an
// MPI implementation's mpi.h is found, so the device library never depends on libmpi.  It
// is never selected implicitly: the caller hands over an MPI communicator explicitly.
#include <mpi.h>

#include <chrono>
#include <cstring>
#include <vector>

#include "comm.hpp"
#include "mpiasyncpools_mpi.h"

namespace mpa {
namespace {

void check(int rc, const char* what) {
  if (rc == MPI_SUCCESS) return;
  char msg[MPI_MAX_ERROR_STRING] = {0};
  int len = 0;
  MPI_Error_string(rc, msg, &len);
  fail(MPA_ERROR, "%s failed: %s", what, msg);
}

class MpiComm final : public Comm {
 public:
  MpiComm(MPI_Comm comm, int64_t nworkers) : Comm(nworkers), comm_(comm), done_(size_t(nworkers), 0) {}

  ~MpiComm() override {
    // requests still in flight belong to a pool that was not drained (waitall!); cancel the
    // receives so MPI_Finalize does not wait on them (the sends complete on their own)
    for (MPI_Request& r : rreq_)
      if (r != MPI_REQUEST_NULL) {
        MPI_Cancel(&r);
        MPI_Request_free(&r);
      }
  }

  int transport() const override { return MPA_TRANSPORT_MPI; }

  void begin_call(const CallBufs& b) override {
    b_ = b;
    if (size_t(b.n) > rreq_.size()) {
      rreq_.resize(size_t(b.n), MPI_REQUEST_NULL);
      sreq_.resize(size_t(b.n), MPI_REQUEST_NULL);
      posted_.resize(size_t(b.n), nullptr);
      rl_.resize(size_t(b.n), 0);
    }
  }

  // :130-138 isendbufs[i] .= sendbuf; Isend; Irecv!
  void post(int64_t i, int64_t rank, int64_t tag) override {
    if (shutdown_) fail(MPA_ERROR, "comm has been shut down");
    const size_t k = size_t(i);
    uint8_t* slot = b_.isendbuf + k * b_.sl;
    if (b_.sl) std::memcpy(slot, b_.sendbuf, b_.sl);
    uint8_t* chunk = b_.irecvbuf + k * b_.rl;
    check(MPI_Isend(slot, int(b_.sl), MPI_BYTE, int(rank), int(tag), comm_, &sreq_[k]), "MPI_Isend");
    check(MPI_Irecv(chunk, int(b_.rl), MPI_BYTE, int(rank), int(tag), comm_, &rreq_[k]), "MPI_Irecv");
    posted_[k] = chunk;
    rl_[k] = b_.rl;
  }

  // :99 Test!(rreqs[i])
  bool test(int64_t i, int64_t rank) override {
    (void)rank;
    int flag = 0;
    check(MPI_Test(&rreq_[size_t(i)], &flag, MPI_STATUS_IGNORE), "MPI_Test");
    return flag != 0;
  }

  // :161 Waitany!(rreqs): completed / never-posted entries are MPI_REQUEST_NULL already
  int64_t waitany(int64_t n, const int64_t* ranks, const uint8_t* live) override {
    (void)ranks;
    (void)live;
    int idx = MPI_UNDEFINED;
    check(MPI_Waitany(int(n), rreq_.data(), &idx, MPI_STATUS_IGNORE), "MPI_Waitany");
    return idx == MPI_UNDEFINED ? -1 : int64_t(idx);
  }

  // :212 Waitall!(rreqs)
  void waitall(int64_t n, const int64_t* ranks, const uint8_t* live) override {
    (void)ranks;
    (void)live;
    check(MPI_Waitall(int(n), rreq_.data(), MPI_STATUSES_IGNORE), "MPI_Waitall");
  }

  // recvbufs[i] .= irecvbufs[i]; Wait!(sreqs[i])  (:108/:113, :167/:171, :216/:218)
  void harvest(int64_t i, int64_t rank) override {
    const size_t k = size_t(i);
    if (posted_[k] && b_.recvbuf) std::memcpy(b_.recvbuf + k * b_.rl, posted_[k], rl_[k] < b_.rl ? rl_[k] : b_.rl);
    check(MPI_Wait(&sreq_[k], MPI_STATUS_IGNORE), "MPI_Wait");
    done_[size_t(rank - 1)] += 1;
  }

  void flush() override {}  // every verb above acts immediately, as in the reference
  void end_call() override {}

  uint64_t now_ns() override {
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now().time_since_epoch())
                        .count());
  }

  int64_t tasks_done(int64_t rank) override { return done_[size_t(rank - 1)]; }

  // the worker programs own their lifecycle (the reference's examples send a control tag,
  // examples/iterative_example.jl:49-52); shutdown only refuses further posts
  void shutdown() override { shutdown_ = true; }

 private:
  MPI_Comm comm_;
  CallBufs b_;
  std::vector<MPI_Request> rreq_, sreq_;
  std::vector<uint8_t*> posted_;
  std::vector<size_t> rl_;
  std::vector<int64_t> done_;
};

}  // namespace
}  // namespace mpa

extern "C" int mpa_comm_create_mpi(int64_t mpi_comm_f, mpa_comm** out) {
  try {
    if (!out) mpa::fail(MPA_ARGUMENT_ERROR, "out is NULL");
    int init = 0;
    MPI_Initialized(&init);
    if (!init) mpa::fail(MPA_ERROR, "MPI is not initialized");
    MPI_Comm comm = MPI_Comm_f2c(MPI_Fint(mpi_comm_f));
    if (comm == MPI_COMM_NULL) mpa::fail(MPA_ARGUMENT_ERROR, "comm is MPI_COMM_NULL");
    int size = 0;
    mpa::check(MPI_Comm_size(comm, &size), "MPI_Comm_size");
    *out = mpa::adopt_comm(new mpa::MpiComm(comm, int64_t(size) - 1));
    return MPA_OK;
  } catch (const mpa::Failure& e) {
    return e.code;
  } catch (...) {
    mpa::set_error("unexpected C++ exception");
    return MPA_ERROR;
  }
}
