// The asyncmap!/waitall! state machine of MPIAsyncPools.jl, restated over the Comm
// transport interface.  Every block cites the reference line it reproduces.
#include "pool.hpp"

namespace mpa {

// src/MPIAsyncPools.jl:35-43, :46
Pool::Pool(int64_t n_, const int64_t* ranks_, int64_t epoch0, int64_t nwait_)
    : n(n_), ranks(size_t(n_)), sepochs(size_t(n_), 0), repochs(size_t(n_), epoch0),
      stimestamps(size_t(n_), 0), active(size_t(n_), 0), rreq_live(size_t(n_), 0), received(size_t(n_), 0),
      latency(size_t(n_), 0.0), nwait(nwait_), epoch(epoch0) {
  for (int64_t i = 0; i < n; ++i) ranks[size_t(i)] = ranks_ ? ranks_[i] : i + 1;
}

namespace {

// recvbufs[i] .= irecvbufs[i]; repochs[i] = sepochs[i] with the latency record
// (:105-109, :164-168, :215-217)
inline void harvest(Pool& p, Comm& c, int64_t i) {
  const size_t k = size_t(i);
  p.latency[k] = double(c.now_ns() - uint64_t(p.stimestamps[k])) / 1e9;
  c.harvest(i, p.ranks[k]);
  p.repochs[k] = p.sepochs[k];
  p.received[k] = 1;
}

// isendbufs[i] .= sendbuf; sepochs; stimestamps; Isend + Irecv! (:130-138, :178-183)
inline void dispatch(Pool& p, Comm& c, int64_t i, int64_t tag) {
  const size_t k = size_t(i);
  p.sepochs[k] = p.epoch;
  p.stimestamps[k] = int64_t(c.now_ns());
  c.post(i, p.ranks[k], tag);
  p.rreq_live[k] = 1;
}

// the gated replay's observation step (gate.cpp); a schedule that fails (kind mismatch,
// over-release, timeout) closes the call first, as every other failure inside a call does
inline void gate_step(Comm& c, int kind) {
  try {
    c.gate(kind);
  } catch (...) {
    c.end_call();
    throw;
  }
}

void check_comm(Pool& p, Comm* comm) {
  if (!comm) fail(MPA_ARGUMENT_ERROR, "comm is NULL");
  for (int64_t i = 0; i < p.n; ++i)
    if (p.ranks[size_t(i)] < 1 || p.ranks[size_t(i)] > comm->nworkers())
      fail(MPA_ARGUMENT_ERROR, "pool rank %lld is not a worker rank of comm (1:%lld)",
           (long long)p.ranks[size_t(i)], (long long)comm->nworkers());
  if (p.comm && p.comm != comm) {
    for (int64_t i = 0; i < p.n; ++i)
      if (p.active[size_t(i)])
        fail(MPA_ARGUMENT_ERROR, "asyncmap!: the pool has outstanding requests on another comm");
  }
  p.comm = comm;
}

}  // namespace

void asyncmap(Pool& p, const AsyncmapArgs& a) {
  const int64_t comm_size = p.n;                                                   // :69
  if (a.nwait_kind == MPA_NWAIT_INT && !(0 <= a.nwait && a.nwait <= comm_size))    // :70-72
    fail(MPA_ARGUMENT_ERROR, "nwait must be in the range [0, length(pool.ranks)], but is %lld",
         (long long)a.nwait);
  // :73-74 (isbitstype) are host-language type checks done by the binding.
  if (a.isend_bytes != size_t(comm_size) * a.send_bytes)                           // :75
    fail(MPA_DIMENSION_MISMATCH,
         "sendbuf is of size %zu bytes, but isendbuf is of size %zu bytes when %zu bytes are needed",
         a.send_bytes, a.isend_bytes, size_t(comm_size) * a.send_bytes);
  if (a.recv_bytes != a.irecv_bytes)                                               // :76
    fail(MPA_DIMENSION_MISMATCH, "recvbuf is of size %zu bytes, but irecvbuf is of size %zu bytes",
         a.recv_bytes, a.irecv_bytes);
  if (comm_size == 0) fail(MPA_ERROR, "DivideError: integer division error");      // mod(x, 0), :77
  if (a.recv_length % size_t(comm_size) != 0)                                      // :77
    fail(MPA_DIMENSION_MISMATCH, "The length of recvbuf and irecvbuf must be a multiple of the number of workers");
  check_comm(p, a.comm);
  Comm& c = *a.comm;

  CallBufs b;                                                                      // :80-84
  b.sendbuf = static_cast<const uint8_t*>(a.sendbuf);
  b.sl = a.send_bytes;
  b.recvbuf = static_cast<uint8_t*>(a.recvbuf);
  b.isendbuf = static_cast<uint8_t*>(a.isendbuf);
  b.irecvbuf = static_cast<uint8_t*>(a.irecvbuf);
  b.rl = a.irecv_bytes / size_t(comm_size);
  b.n = comm_size;
  b.await_all = a.nwait_kind == MPA_NWAIT_INT && a.nwait == comm_size;
  c.begin_call(b);

  p.epoch = a.epoch;                                                               // :87
  gate_step(c, MPA_GATE_CALL);  // gated replay: the completions phase 1's Test! may see (gate.cpp)

  for (int64_t i = 0; i < comm_size; ++i) {                                        // :91-114
    const size_t k = size_t(i);
    if (!p.active[k]) continue;                                                    // :94-96
    if (!c.test(i, p.ranks[k])) continue;                                          // :99-102
    p.rreq_live[k] = 0;
    harvest(p, c, i);                                                              // :105-109
    p.active[k] = 0;                                                               // :110
  }                                                                                // :113 Wait!(sreq): no-op

  // owed[i]: worker i was sent this epoch's message in phase 2 and has not replied (a
  // transport hint only: set_wait_hold below; the state machine does not read it)
  std::vector<uint8_t> owed(size_t(comm_size), 0);
  int64_t nowed = 0;
  for (int64_t i = 0; i < comm_size; ++i) {                                        // :118-139
    const size_t k = size_t(i);
    if (p.active[k]) continue;                                                     // :121-123
    p.active[k] = 1;                                                               // :126
    dispatch(p, c, i, a.tag);                                                      // :130-138
    owed[k] = 1;
    ++nowed;
  }
  c.flush();  // phase-1 copies, then the sends of phase 2, in the reference's order

  int64_t nrecv = 0;                                                               // :145
  for (;;) {
    if (a.nwait_kind == MPA_NWAIT_INT) {                                           // :148-151
      if (nrecv >= a.nwait) break;
    } else if (a.nwait_kind == MPA_NWAIT_FN) {                                     // :152-155
      const int r = a.fn(a.fn_ctx, p.epoch, p.repochs.data(), comm_size);
      if (r < 0) { c.end_call(); fail(MPA_CALLBACK_ERROR, "nwait function raised an exception"); }
      if (r) break;
    } else {                                                                       // :156-158
      c.end_call();
      fail(MPA_ERROR, "nwait must be either an Integer or a Function, but is a %s",
           a.nwait_typename ? a.nwait_typename : "?");
    }
    c.set_wait_hold(a.nwait_kind == MPA_NWAIT_INT && nowed >= a.nwait - nrecv);
    if (c.gated()) {  // the completions this Waitany! may see (a call that finds none live is MPI_UNDEFINED)
      bool live = false;
      for (int64_t j = 0; j < comm_size; ++j) live |= p.rreq_live[size_t(j)] != 0;
      if (live) gate_step(c, MPA_GATE_WAIT);
    }
    const int64_t i = c.waitany(comm_size, p.ranks.data(), p.rreq_live.data());   // :161
    if (i < 0) {  // MPI_UNDEFINED: undefined in the reference; an error here
      c.end_call();
      fail(MPA_ERROR, "asyncmap!: no outstanding requests and the nwait condition is unsatisfiable");
    }
    const size_t k = size_t(i);
    p.rreq_live[k] = 0;
    if (owed[k]) {
      owed[k] = 0;
      --nowed;
    }
    harvest(p, c, i);                                                              // :164-168
    if (p.repochs[k] == p.epoch) {                                                 // :174-176
      nrecv += 1;
      p.active[k] = 0;
    } else {                                                                       // :177-184
      dispatch(p, c, i, a.tag);
      c.flush_stale();  // the stale chunk must reach recvbuf before the worker overwrites it
    }
  }
  c.end_call();
}                                                                                  // :187

void waitall(Pool& p, void* recvbuf, size_t recv_bytes, size_t recv_length, void* irecvbuf,
             size_t irecv_bytes) {
  const int64_t comm_size = p.n;                                                   // :196
  if (recv_bytes != irecv_bytes)                                                   // :198
    fail(MPA_DIMENSION_MISMATCH, "recvbuf is of size %zu bytes, but irecvbuf is of size %zu bytes",
         recv_bytes, irecv_bytes);
  if (comm_size == 0) fail(MPA_ERROR, "DivideError: integer division error");      // mod(x, 0), :199
  if (recv_length % size_t(comm_size) != 0)                                        // :199
    fail(MPA_DIMENSION_MISMATCH, "The length of recvbuf and irecvbuf must be a multiple of the number of workers");
  int64_t nactive = 0;                                                             // :201-204
  for (int64_t i = 0; i < comm_size; ++i) nactive += p.active[size_t(i)];
  if (nactive == 0) return;
  Comm& c = *p.comm;
  CallBufs b;                                                                      // :207-209
  b.recvbuf = static_cast<uint8_t*>(recvbuf);
  b.irecvbuf = static_cast<uint8_t*>(irecvbuf);
  b.rl = irecv_bytes / size_t(comm_size);
  b.n = comm_size;
  c.begin_call(b);
  gate_step(c, MPA_GATE_WAITALL);
  c.waitall(comm_size, p.ranks.data(), p.rreq_live.data());                        // :212
  for (int64_t i = 0; i < comm_size; ++i) {                                        // :213-221
    const size_t k = size_t(i);
    if (p.active[k]) {
      p.rreq_live[k] = 0;
      harvest(p, c, i);
      p.active[k] = 0;
    }
  }
  c.end_call();
}                                                                                  // :223

}  // namespace mpa
