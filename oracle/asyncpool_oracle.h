/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of MPIAsyncPools.jl (severinson/MPIStragglers.jl, package
 * `MPIAsyncPools` v0.1.0), used as the parity checker for the MI355X build.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product library (mpistragglers.jl_amd/) never links or calls it.
 *
 * What is restated (reference file:line):
 *   orc_pool_create   src/MPIAsyncPools.jl:35-46   (MPIAsyncPool ctor)
 *   orc_asyncmap      src/MPIAsyncPools.jl:68-188  (Base.asyncmap!)
 *   orc_waitall       src/MPIAsyncPools.jl:195-224 (waitall!)
 * The MPI point-to-point layer (MPI.jl -> libmpi, not vendored, Project.toml:7,10) is
 * abstracted as orc_transport.  Two transports exist:
 *   - orc_sim:   a discrete-event, virtual-clock restatement of the worker protocol of
 *                examples/iterative_example.jl:55-82 / test/kmap1.jl:23-33 /
 *                test/kmap2.jl:76-99 with a seeded per-(worker, task) delay schedule.
 *   - the threaded CPU baseline in cpu_baseline.c (real clock, real compute).
 *
 * Parity status: the reference is Julia + MPI.jl, neither of which exists in this
 * image, so the oracle cannot be run against the reference itself.  It is pinned by the
 * reference's own known-answer / property tests (test/kmap1.jl:22,30;
 * test/kmap2.jl:22,50,53,60,70,71), restated in tests/test_oracle.py.  MPI_Waitany
 * tie order (several requests complete) is not pinned by any reference test: this
 * oracle defines it as lowest index first (the order MPICH's array scan returns).
 */
#ifndef MPA_ASYNCPOOL_ORACLE_H
#define MPA_ASYNCPOOL_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  ORC_OK = 0,
  ORC_ARGUMENT_ERROR = 1,  /* Julia ArgumentError */
  ORC_DIMENSION_MISMATCH = 2,  /* Julia DimensionMismatch */
  ORC_ERROR = 3,  /* Julia error(...) / ErrorException */
};

/* MPI point-to-point abstraction; indices are 0-based pool positions. */
typedef struct orc_transport {
  void* ctx;
  /* MPI.Isend(isendbufs[i], rank, tag, comm) + MPI.Irecv!(irecvbufs[i], rank, tag, comm) */
  void (*isend_irecv)(void* ctx, int64_t i, int64_t rank, const uint8_t* sbuf, size_t sl,
                      uint8_t* rbuf, size_t rl, int64_t tag);
  /* MPI.Test!(rreqs[i]) -> 1 if complete (the reply is then in rbuf) */
  int (*test)(void* ctx, int64_t i);
  /* MPI.Waitany!(rreqs): live[i] != 0 marks non-null requests; returns i or -1 */
  int64_t (*waitany)(void* ctx, int64_t n, const uint8_t* live);
  /* MPI.Waitall!(rreqs) */
  void (*waitall)(void* ctx, int64_t n, const uint8_t* live);
  /* Base.time_ns() */
  uint64_t (*time_ns)(void* ctx);
  /* optional (NULL = none): the call's observation point before phase 1, ORC_OBS_CALL; the
   * observation points of Waitany!/Waitall! are the transport's own calls above */
  void (*observe)(void* ctx, int kind);
} orc_transport;

/* observation points of the state machine (the step kinds of a gated replay schedule,
 * include/mpiasyncpools.h MPA_GATE_*), plus the post records of the sim's log */
enum { ORC_OBS_CALL = 0, ORC_OBS_WAIT = 1, ORC_OBS_WAITALL = 2, ORC_OBS_POST = 3 };

typedef struct orc_pool {
  int64_t n;
  int64_t* ranks;       /* :25 */
  int64_t* sepochs;     /* :28 */
  int64_t* repochs;     /* :29 */
  uint8_t* active;      /* :30 */
  int64_t* stimestamps; /* :31 */
  double* latency;      /* :32 */
  uint8_t* rreq_live;   /* MPI request handle non-null (:26-27) */
  int64_t nwait;        /* :33 */
  int64_t epoch;        /* :34 */
  char errmsg[512];
} orc_pool;

/* nwait as Function: nwait(epoch, repochs)::Bool (:153).  Return 0/1. */
typedef int (*orc_nwait_fn)(void* ctx, int64_t epoch, const int64_t* repochs, int64_t n);

enum { ORC_NWAIT_INT = 0, ORC_NWAIT_FN = 1, ORC_NWAIT_OTHER = 2 };

orc_pool* orc_pool_create(int64_t n, const int64_t* ranks, int64_t epoch0, int64_t nwait);
void orc_pool_destroy(orc_pool* p);

int orc_asyncmap(orc_pool* p, const orc_transport* tp,
                 const uint8_t* sendbuf, size_t send_bytes,
                 uint8_t* recvbuf, size_t recv_bytes, size_t recv_len,
                 uint8_t* isendbuf, size_t isend_bytes,
                 uint8_t* irecvbuf, size_t irecv_bytes,
                 int nwait_kind, int64_t nwait, orc_nwait_fn fn, void* fn_ctx,
                 const char* nwait_typename, int64_t epoch, int64_t tag);

int orc_waitall(orc_pool* p, const orc_transport* tp,
                uint8_t* recvbuf, size_t recv_bytes, size_t recv_len,
                uint8_t* irecvbuf, size_t irecv_bytes);

/* ---------------- virtual-clock simulated worker transport ---------------- */
enum {
  ORC_WORKER_ECHO = 0,   /* reply = received bytes (truncated / zero padded) */
  ORC_WORKER_KMAP1 = 1,  /* reply[0] = Float64(rank)              test/kmap1.jl:24-32 */
  ORC_WORKER_KMAP2 = 2,  /* reply = Float64[rank, t, epoch]        test/kmap2.jl:76-99 */
  ORC_WORKER_TAG = 3,    /* reply = Int64[rank, t, first 8 bytes]  (trace tagging) */
};

typedef struct orc_sim orc_sim;
/* durations_ns: [nworkers][ncols] task durations; task t (1-based) of worker w uses
 * durations_ns[w*ncols + (t-1) % ncols].  compute_ns is added to every task. */
orc_sim* orc_sim_create(int64_t nworkers, int kind, const int64_t* durations_ns, int64_t ncols,
                        int64_t compute_ns);
void orc_sim_destroy(orc_sim* s);
void orc_sim_transport(orc_sim* s, orc_transport* out);
void orc_sim_advance(orc_sim* s, int64_t dt_ns);
int64_t orc_sim_now(const orc_sim* s);
int64_t orc_sim_tasks(const orc_sim* s, int64_t worker);

/* event trace of the simulated transport, for fixtures: one record per completion
 * observed by the coordinator */
typedef struct { int64_t worker, t, post_ns, done_ns, seen_ns; } orc_event;
int64_t orc_sim_events(const orc_sim* s, orc_event* out, int64_t cap);

/* observation log of the simulated transport, in program order: ORC_OBS_POST for every
 * task posted (worker, t, done_ns), ORC_OBS_CALL / _WAIT / _WAITALL for every observation
 * point with the virtual time it observes (now; a Waitany! that blocks logs the time it
 * advances to, one that finds no live request logs nothing).  The completions an
 * observation sees are exactly the posted tasks with done_ns <= now: the gate schedule of a
 * device replay (oracle/oracle.py gate_schedule). */
typedef struct { int64_t kind, worker, t, done_ns, now; } orc_obs;
int64_t orc_sim_obs(const orc_sim* s, orc_obs* out, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
