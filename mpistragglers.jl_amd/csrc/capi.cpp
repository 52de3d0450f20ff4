// extern "C" entry points declared in include/mpiasyncpools.h.  Every entry converts
// library failures into a status code + thread-local message (mpa_last_error).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <new>
#include <string>

#include "comm.hpp"
#include "hip_transport.hpp"
#include "kernels.hpp"
#include "pool.hpp"

#ifndef MPA_MEASURE
#define MPA_MEASURE 0
#endif

namespace mpa {
void sim_set_compute(Comm* c, int64_t ns);
void sim_advance(Comm* c, int64_t dt);
int64_t sim_now(const Comm* c);
void hip_set_stream(Comm* c, void* s);
void* hip_get_stream(Comm* c);
void hip_set_timing(Comm* c, int period);
void hip_timing(Comm* c, double out[4]);
void hip_exchange_timing(Comm* c, double out[3]);
void hip_set_trace(Comm* c, int64_t capacity);
int64_t hip_read_trace(Comm* c, int64_t* out, int64_t capacity);
extern int g_lsq_grid;
Comm* make_dist_comm(int64_t nworkers, const int* placement, int my_rank, const char* shm_name, size_t max_msg);
void hip_serve(Comm* c);
void hip_pause_servers(Comm* c);
void hip_set_defer_end(Comm* c, bool on, bool prearm_ok = false);
void hip_stage_update(Comm* c, int dtype, int64_t elems, const double* w, int64_t n, double eta, void* x, void* mirror,
                      bool msg_bf16);
void hip_set_ahead(Comm* c, int64_t left, int dtype, int64_t elems, const double* w, int64_t n, double eta, void* x,
                   void* mirror, bool msg_bf16);
void hip_flush(Comm* c);
int hip_payload_path(Comm* c, int64_t rank);
Comm* make_host_dist_comm(int64_t nworkers, const int* placement, int my_rank, const char* shm_name, size_t max_msg);
void host_serve(Comm* c);
void host_pause_servers(Comm* c);
}  // namespace mpa

struct mpa_pool {
  mpa::Pool p;
};
struct mpa_comm {
  mpa::Comm* c;
};

mpa_comm* mpa::adopt_comm(mpa::Comm* c) { return new mpa_comm{c}; }

namespace {

template <typename F>
int guarded(F&& f) {
  try {
    f();
    return MPA_OK;
  } catch (const mpa::Failure& e) {
    return e.code;
  } catch (const std::bad_alloc&) {
    mpa::set_error("out of host memory");
    return MPA_ERROR;
  } catch (...) {
    mpa::set_error("unexpected C++ exception");
    return MPA_ERROR;
  }
}

mpa::Comm& comm_of(mpa_comm* c) {
  if (!c || !c->c) mpa::fail(MPA_ARGUMENT_ERROR, "comm is NULL");
  return *c->c;
}

void need_hip(mpa::Comm& c) {
  if (c.transport() != MPA_TRANSPORT_HIP) mpa::fail(MPA_ARGUMENT_ERROR, "this call needs a HIP-transport comm");
}

#define HIPCHECK_C(expr)                                                                        \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) mpa::fail(MPA_DEVICE_ERROR, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

}  // namespace

extern "C" {

int mpa_abi_version(void) { return MPA_ABI_VERSION; }
const char* mpa_last_error(void) { return mpa::last_error(); }
int mpa_tune(const char* key, int64_t value) {
  return guarded([&] {
    const std::string k = key ? key : "";
    if (k == "lsq_variant") {
      if (mpa::lsq_set_variant(int(value)) < 0) mpa::fail(MPA_ARGUMENT_ERROR, "no lsq variant %lld", (long long)value);
    } else if (k == "lsq_grid") {
      if (value < 0 || value > (1 << 20)) mpa::fail(MPA_ARGUMENT_ERROR, "bad lsq_grid");
      mpa::g_lsq_grid = int(value);
    } else {
      mpa::fail(MPA_ARGUMENT_ERROR, "unknown tuning key '%s'", k.c_str());
    }
  });
}

const char* mpa_build_info(void) {
  static std::string info = std::string("gfx950; lsq c2 variant: ") + mpa::lsq_variant_name() +
                            (MPA_MEASURE ? "; measurement build (MEASURE=1)" : "");
  return info.c_str();
}

int mpa_pool_create(int64_t n, const int64_t* ranks, int64_t epoch0, int64_t nwait, mpa_pool** out) {
  return guarded([&] {
    if (!out) mpa::fail(MPA_ARGUMENT_ERROR, "out is NULL");
    if (n < 0) mpa::fail(MPA_ARGUMENT_ERROR, "n must be non-negative");
    *out = new mpa_pool{mpa::Pool(n, ranks, epoch0, nwait)};
  });
}

void mpa_pool_destroy(mpa_pool* pool) { delete pool; }
int64_t mpa_pool_size(const mpa_pool* pool) { return pool ? pool->p.n : 0; }
int64_t* mpa_pool_ranks(mpa_pool* pool) { return pool->p.ranks.data(); }
int64_t* mpa_pool_sepochs(mpa_pool* pool) { return pool->p.sepochs.data(); }
int64_t* mpa_pool_repochs(mpa_pool* pool) { return pool->p.repochs.data(); }
uint8_t* mpa_pool_active(mpa_pool* pool) { return pool->p.active.data(); }
int64_t* mpa_pool_stimestamps(mpa_pool* pool) { return pool->p.stimestamps.data(); }
double* mpa_pool_latency(mpa_pool* pool) { return pool->p.latency.data(); }
int64_t* mpa_pool_nwait(mpa_pool* pool) { return &pool->p.nwait; }
int64_t* mpa_pool_epoch(mpa_pool* pool) { return &pool->p.epoch; }

int mpa_asyncmap(mpa_pool* pool, const void* sendbuf, size_t sendbuf_bytes, void* recvbuf, size_t recvbuf_bytes,
                 size_t recvbuf_length, void* isendbuf, size_t isendbuf_bytes, void* irecvbuf,
                 size_t irecvbuf_bytes, mpa_comm* comm, int nwait_kind, int64_t nwait, mpa_nwait_fn nwait_fn,
                 void* nwait_ctx, const char* nwait_typename, int64_t epoch, int64_t tag, int64_t** repochs_out) {
  return guarded([&] {
    if (!pool) mpa::fail(MPA_ARGUMENT_ERROR, "pool is NULL");
    if (nwait_kind == MPA_NWAIT_FN && !nwait_fn) mpa::fail(MPA_ARGUMENT_ERROR, "nwait function is NULL");
    mpa::AsyncmapArgs a{sendbuf, sendbuf_bytes, recvbuf, recvbuf_bytes, recvbuf_length, isendbuf, isendbuf_bytes,
                        irecvbuf, irecvbuf_bytes, comm ? comm->c : nullptr, nwait_kind, nwait, nwait_fn,
                        nwait_ctx, nwait_typename, epoch, tag};
    mpa::asyncmap(pool->p, a);
    if (repochs_out) *repochs_out = pool->p.repochs.data();
  });
}

int mpa_waitall(mpa_pool* pool, void* recvbuf, size_t recvbuf_bytes, size_t recvbuf_length, void* irecvbuf,
                size_t irecvbuf_bytes, int64_t** repochs_out) {
  return guarded([&] {
    if (!pool) mpa::fail(MPA_ARGUMENT_ERROR, "pool is NULL");
    mpa::waitall(pool->p, recvbuf, recvbuf_bytes, recvbuf_length, irecvbuf, irecvbuf_bytes);
    if (repochs_out) *repochs_out = pool->p.repochs.data();
  });
}

int mpa_comm_create(int transport, int64_t nworkers, const int* devices, mpa_comm** out) {
  return guarded([&] {
    if (!out) mpa::fail(MPA_ARGUMENT_ERROR, "out is NULL");
    if (nworkers < 0) mpa::fail(MPA_ARGUMENT_ERROR, "nworkers must be non-negative");
    mpa::Comm* c = nullptr;
    if (transport == MPA_TRANSPORT_HIP) c = mpa::make_hip_comm(nworkers, devices);
    else if (transport == MPA_TRANSPORT_SIM) c = mpa::make_sim_comm(nworkers);
    else mpa::fail(MPA_ARGUMENT_ERROR, "unknown transport %d", transport);
    *out = new mpa_comm{c};
  });
}

int mpa_comm_create_dist(int transport, int64_t nworkers, const int* placement, int my_rank, const char* shm_name,
                         size_t max_msg_bytes, mpa_comm** out) {
  return guarded([&] {
    if (!out) mpa::fail(MPA_ARGUMENT_ERROR, "out is NULL");
    if (nworkers < 0 || my_rank < 0) mpa::fail(MPA_ARGUMENT_ERROR, "bad nworkers / rank");
    mpa::Comm* c = nullptr;
    if (transport == MPA_TRANSPORT_HIP) c = mpa::make_dist_comm(nworkers, placement, my_rank, shm_name, max_msg_bytes);
    else if (transport == MPA_TRANSPORT_HOST) c = mpa::make_host_dist_comm(nworkers, placement, my_rank, shm_name, max_msg_bytes);
    else mpa::fail(MPA_ARGUMENT_ERROR, "multi-process communicators are MPA_TRANSPORT_HIP or MPA_TRANSPORT_HOST");
    *out = new mpa_comm{c};
  });
}

int mpa_comm_serve(mpa_comm* comm) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    if (c.transport() == MPA_TRANSPORT_HIP) mpa::hip_serve(&c);
    else if (c.transport() == MPA_TRANSPORT_HOST) mpa::host_serve(&c);
    else mpa::fail(MPA_ARGUMENT_ERROR, "not a multi-process communicator");
  });
}

int mpa_comm_payload_path(mpa_comm* comm, int64_t rank) {
  if (!comm || !comm->c || comm->c->transport() != MPA_TRANSPORT_HIP) return 0;
  return mpa::hip_payload_path(comm->c, rank);
}

int mpa_comm_pause_servers(mpa_comm* comm) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    if (c.transport() == MPA_TRANSPORT_HIP) mpa::hip_pause_servers(&c);
    else if (c.transport() == MPA_TRANSPORT_HOST) mpa::host_pause_servers(&c);
    else mpa::fail(MPA_ARGUMENT_ERROR, "not a multi-process communicator");
  });
}

void mpa_comm_destroy(mpa_comm* comm) {
  if (!comm) return;
  delete comm->c;
  delete comm;
}

int64_t mpa_comm_size(const mpa_comm* comm) { return comm && comm->c ? comm->c->nworkers() + 1 : 0; }

int mpa_comm_set_stream(mpa_comm* comm, void* stream) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    need_hip(c);
    mpa::hip_set_stream(&c, stream);
  });
}

int mpa_comm_set_task_kmap(mpa_comm* comm, int64_t rank, int task) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    if (task != MPA_TASK_ECHO && task != MPA_TASK_KMAP1 && task != MPA_TASK_KMAP2)
      mpa::fail(MPA_ARGUMENT_ERROR, "task must be MPA_TASK_ECHO, MPA_TASK_KMAP1 or MPA_TASK_KMAP2");
    mpa::TaskSpec& t = c.task(rank);
    const mpa::TaskSpec saved = t;
    t.kind = task;
    try {
      c.on_task_changed(rank);
    } catch (...) {
      t = saved;
      throw;
    }
  });
}

int mpa_comm_set_task_lsq(mpa_comm* comm, int64_t rank, int dtype, int64_t rows, int64_t cols, const void* A,
                          int64_t lda, const void* b) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    need_hip(c);
    if (dtype != MPA_F32 && dtype != MPA_F64) mpa::fail(MPA_ARGUMENT_ERROR, "least squares: dtype must be F32 or F64");
    if (rows < 0 || cols <= 0) mpa::fail(MPA_ARGUMENT_ERROR, "least squares: bad shape");
    if (rows > 0 && (!A || !b)) mpa::fail(MPA_ARGUMENT_ERROR, "least squares: A and b must be device pointers");
    mpa::TaskSpec& t = c.task(rank);
    const mpa::TaskSpec saved = t;
    t.kind = MPA_TASK_LSQ;
    t.dtype = dtype;
    t.rows = rows;
    t.cols = cols;
    t.lda = lda;
    t.A = A;
    t.b = b;
    try {
      c.on_task_changed(rank);
    } catch (...) {
      t = saved;
      throw;
    }
  });
}

int mpa_comm_set_task_lsq_batch(mpa_comm* comm, int64_t rank, int64_t rows, int64_t cols, int64_t k, const void* A,
                                int64_t lda, const void* B) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    need_hip(c);
    if (rows < 0 || cols <= 0 || k <= 0) mpa::fail(MPA_ARGUMENT_ERROR, "batched least squares: bad shape");
    if (rows > 0 && (!A || !B)) mpa::fail(MPA_ARGUMENT_ERROR, "batched least squares: A and B must be device pointers");
    mpa::TaskSpec& t = c.task(rank);
    const mpa::TaskSpec saved = t;
    t.kind = MPA_TASK_LSQ_BATCH;
    t.dtype = MPA_BF16;
    t.rows = rows;
    t.cols = cols;
    t.k = k;
    t.lda = lda;
    t.A = A;
    t.b = B;
    try {
      c.on_task_changed(rank);
    } catch (...) {
      t = saved;
      throw;
    }
  });
}

int mpa_comm_set_delays(mpa_comm* comm, int64_t rank, const int64_t* delays_ns, int64_t count) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    if (count < 0 || (count > 0 && !delays_ns)) mpa::fail(MPA_ARGUMENT_ERROR, "bad delay schedule");
    for (int64_t k = 0; k < count; ++k)
      if (delays_ns[k] < 0) mpa::fail(MPA_ARGUMENT_ERROR, "delays must be non-negative");
    c.task(rank).delays_ns.assign(delays_ns, delays_ns + count);
    c.on_delays_changed(rank);
  });
}

int64_t mpa_comm_tasks_done(mpa_comm* comm, int64_t rank) {
  int64_t r = -1;
  const int rc = guarded([&] {
    mpa::Comm& c = comm_of(comm);
    c.task(rank);
    r = c.tasks_done(rank);
  });
  return rc == MPA_OK ? r : -1;
}

int mpa_comm_shutdown(mpa_comm* comm) {
  return guarded([&] { comm_of(comm).shutdown(); });
}

int mpa_comm_set_gate(mpa_comm* comm, int64_t nsteps, const int* kinds, const int64_t* offsets, const int64_t* ranks) {
  return guarded([&] { comm_of(comm).set_gate(kinds, offsets, ranks, nsteps); });
}

int64_t mpa_comm_counter(mpa_comm* comm, const char* name) {
  int64_t r = -1;
  const int rc = guarded([&] {
    if (!name) mpa::fail(MPA_ARGUMENT_ERROR, "name is NULL");
    r = comm_of(comm).counter(name);
  });
  return rc == MPA_OK ? r : -1;
}

int mpa_comm_set_timing(mpa_comm* comm, int enable) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    need_hip(c);
    if (enable < 0) mpa::fail(MPA_ARGUMENT_ERROR, "enable < 0");
    mpa::hip_set_timing(&c, enable);
  });
}

int mpa_comm_timing(mpa_comm* comm, double out[4]) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    need_hip(c);
    if (!out) mpa::fail(MPA_ARGUMENT_ERROR, "out is NULL");
    mpa::hip_timing(&c, out);
  });
}

int mpa_comm_exchange_timing(mpa_comm* comm, double out[3]) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    need_hip(c);
    if (!out) mpa::fail(MPA_ARGUMENT_ERROR, "out is NULL");
    mpa::hip_exchange_timing(&c, out);
  });
}

int mpa_comm_set_trace(mpa_comm* comm, int64_t capacity) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    need_hip(c);
    mpa::hip_set_trace(&c, capacity);
  });
}

int mpa_comm_trace(mpa_comm* comm, int64_t* out, int64_t capacity, int64_t* count) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    need_hip(c);
    if (!count || capacity < 0 || (capacity > 0 && !out)) mpa::fail(MPA_ARGUMENT_ERROR, "bad trace buffer");
    *count = mpa::hip_read_trace(&c, out, capacity);
  });
}

int mpa_comm_sim_set_compute(mpa_comm* comm, int64_t compute_ns) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    if (c.transport() != MPA_TRANSPORT_SIM) mpa::fail(MPA_ARGUMENT_ERROR, "not a SIM comm");
    mpa::sim_set_compute(&c, compute_ns);
  });
}

int mpa_comm_sim_advance(mpa_comm* comm, int64_t dt_ns) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    if (c.transport() != MPA_TRANSPORT_SIM) mpa::fail(MPA_ARGUMENT_ERROR, "not a SIM comm");
    mpa::sim_advance(&c, dt_ns);
  });
}

int64_t mpa_comm_sim_now(const mpa_comm* comm) {
  if (!comm || !comm->c || comm->c->transport() != MPA_TRANSPORT_SIM) return -1;
  return mpa::sim_now(comm->c);
}

static int aggregate_impl(mpa_comm* comm, int dtype, const void* recvbuf, int64_t n, int64_t elems,
                          const double* weights, void* out, int update, double eta, void* mirror = nullptr) {
  return guarded([&] {
    mpa::Comm& c = comm_of(comm);
    need_hip(c);
    if (dtype != MPA_F32 && dtype != MPA_F64) mpa::fail(MPA_ARGUMENT_ERROR, "aggregate: dtype must be F32 or F64");
    if (n < 0 || n > mpa::kMaxAggregate) mpa::fail(MPA_ARGUMENT_ERROR, "aggregate: 0 <= nchunks <= %d", mpa::kMaxAggregate);
    if (elems < 0 || (n > 0 && !weights) || !out || (n > 0 && !recvbuf))
      mpa::fail(MPA_ARGUMENT_ERROR, "aggregate: bad arguments");
    mpa::AggregateArgs a{};
    a.chunks = recvbuf;
    a.out = out;
    a.n = n;
    a.elems = elems;
    a.stride = elems;
    a.eta = eta;
    a.update = update;
    a.mirror = static_cast<uint16_t*>(mirror);
    for (int64_t i = 0; i < n; ++i) a.w[i] = weights[i];
    HIPCHECK_C(mpa::launch_aggregate(dtype, a, static_cast<hipStream_t>(mpa::hip_get_stream(&c))));
  });
}

int mpa_aggregate(mpa_comm* comm, int dtype, const void* recvbuf, int64_t nchunks, int64_t chunk_elems,
                  const double* weights, void* out) {
  return aggregate_impl(comm, dtype, recvbuf, nchunks, chunk_elems, weights, out, 0, 0.0);
}

int mpa_lsq_update(mpa_comm* comm, int dtype, void* x, const void* recvbuf, int64_t nchunks, int64_t cols,
                   const double* weights, double eta) {
  return aggregate_impl(comm, dtype, recvbuf, nchunks, cols, weights, x, 1, eta);
}

}  // extern "C"
namespace {
bool env_off(const char* name) {
  const char* e = std::getenv(name);
  return e && *e == '0';
}

// The iterate update of a descent loop: x -= eta * sum_i w_i chunk_i (fp32 / fp64 x and
// chunks); the message sent to the workers is x itself, or its bf16 mirror (batched variant).
struct DescentUpdate {
  int dtype;
  int64_t elems;
  double eta;
  void* x;
  void* mirror;
  bool msg_bf16;
};

// The coordinator loop shared by mpa_lsq_descent / mpa_lsqb_descent: `epochs` iterations of
// asyncmap! followed by the iterate update (examples/iterative_example.jl:37-47).  The
// update is staged into the next flush (one fused epoch kernel: harvests + update +
// dispatch copies + doorbells), and with integer nwait == n the next epoch is enqueued
// ahead while this one's waits run (HipComm::set_ahead).  MPA_FUSE=0 runs
// the update as its own launch after every call, MPA_AHEAD=0 disables launch-ahead.
int descent_loop(mpa_pool* pool, mpa_comm* comm, const void* msg, size_t msg_bytes, size_t reply_es, void* recvbuf,
                 size_t recvbuf_bytes, void* isendbuf, size_t isendbuf_bytes, void* irecvbuf, size_t irecvbuf_bytes,
                 int nwait_kind, int64_t nwait, mpa_nwait_fn nwait_fn, void* nwait_ctx, double stale_weight,
                 int64_t epochs, const DescentUpdate& up) {
  mpa::Pool& p = pool->p;
  const int64_t n = p.n;
  const int64_t elems = up.elems;
  const size_t rl = size_t(elems) * reply_es;
  int rc = guarded([&] {
    if (!comm || !comm->c) mpa::fail(MPA_ARGUMENT_ERROR, "comm is NULL");
    need_hip(*comm->c);
    // the buffers as the caller sized them: asyncmap!'s own checks (src/MPIAsyncPools.jl:75-77)
    // run on these sizes, and the reply chunks must be the iterate's shape
    if (!recvbuf || !isendbuf || !irecvbuf) mpa::fail(MPA_ARGUMENT_ERROR, "descent: recvbuf, isendbuf and irecvbuf must be given");
    if (isendbuf_bytes != size_t(n) * msg_bytes)
      mpa::fail(MPA_DIMENSION_MISMATCH,
                "sendbuf is of size %zu bytes, but isendbuf is of size %zu bytes when %zu bytes are needed", msg_bytes,
                isendbuf_bytes, size_t(n) * msg_bytes);
    if (recvbuf_bytes != irecvbuf_bytes)
      mpa::fail(MPA_DIMENSION_MISMATCH, "recvbuf is of size %zu bytes, but irecvbuf is of size %zu bytes", recvbuf_bytes,
                irecvbuf_bytes);
    if (recvbuf_bytes != size_t(n) * rl)
      mpa::fail(MPA_DIMENSION_MISMATCH, "descent: recvbuf is of size %zu bytes, but %lld chunks of %zu bytes are needed",
                recvbuf_bytes, (long long)n, rl);
  });
  if (rc != MPA_OK) return rc;
  mpa::Comm* c = comm->c;
  const bool fuse = !env_off("MPA_FUSE");
  const char* tr = std::getenv("MPA_DESCENT_TRACE");  // repochs after every call, to stderr
  const bool trace = tr && *tr == '1';
  const bool ahead = fuse && !env_off("MPA_AHEAD") && nwait_kind == MPA_NWAIT_INT && nwait == n;
  std::vector<double> w(static_cast<size_t>(n), 0.0);
  const std::vector<double> w_all(static_cast<size_t>(n), 1.0);  // every chunk fresh
  struct Restore {
    mpa::Comm* c;
    bool on;
    ~Restore() {
      if (on) mpa::hip_set_defer_end(c, false);
    }
  } restore{c, fuse};
  // pre-armed launches wait on the GPU for the host's next decision: only where nothing but
  // native code runs between two calls (an integer nwait or the native first_plus predicate; a
  // caller's predicate could touch the GPU and wait behind the armed launch)
  const bool prearm_ok = nwait_kind == MPA_NWAIT_INT || (nwait_kind == MPA_NWAIT_FN && nwait_fn == &mpa_nwait_first_plus);
  if (fuse) mpa::hip_set_defer_end(c, true, prearm_ok);
  for (int64_t e = 0; e < epochs; ++e) {
    if (ahead) {
      rc = guarded([&] {
        mpa::hip_set_ahead(c, epochs - 1 - e, up.dtype, elems, w_all.data(), n, up.eta, up.x, up.mirror, up.msg_bf16);
      });
      if (rc != MPA_OK) return rc;
    }
    {
      MPA_HPROF(mpa::kHpAsyncmap);
      rc = mpa_asyncmap(pool, msg, msg_bytes, recvbuf, recvbuf_bytes, recvbuf_bytes / reply_es, isendbuf, isendbuf_bytes,
                        irecvbuf, irecvbuf_bytes, comm, nwait_kind, nwait, nwait_fn, nwait_ctx, "Int64", p.epoch + 1, 0,
                        nullptr);
    }
    if (rc != MPA_OK) return rc;
    if (trace) {
      std::fprintf(stderr, "[mpa descent] epoch %lld repochs", (long long)p.epoch);
      for (int64_t i = 0; i < n; ++i) std::fprintf(stderr, " %lld", (long long)p.repochs[size_t(i)]);
      std::fprintf(stderr, " | sepochs");
      for (int64_t i = 0; i < n; ++i) std::fprintf(stderr, " %lld", (long long)p.sepochs[size_t(i)]);
      std::fprintf(stderr, " | latency ms");
      for (int64_t i = 0; i < n; ++i) std::fprintf(stderr, " %.1f", p.latency[size_t(i)] * 1e3);
      std::fprintf(stderr, "\n");
    }
    double sum = 0;
    for (int64_t i = 0; i < n; ++i) {
      // fresh: weight 1; an older result: stale_weight; nothing received yet (the chunk is
      // unfilled; test/kmap2.jl:42 skips such workers): 0
      const int64_t r = p.repochs[size_t(i)];
      w[size_t(i)] = r == p.epoch ? 1.0 : (p.received[size_t(i)] ? stale_weight : 0.0);
      sum += w[size_t(i)];
    }
    const double s = sum > 0 ? double(n) / sum : 0.0;
    for (auto& v : w) v *= s;
    if (fuse) {
      MPA_HPROF(mpa::kHpUpdate);
      rc = guarded([&] {
        mpa::hip_stage_update(c, up.dtype, elems, w.data(), n, up.eta, up.x, up.mirror, up.msg_bf16);
      });
    } else {
      rc = aggregate_impl(comm, up.dtype, recvbuf, n, elems, w.data(), up.x, 1, up.eta, up.mirror);
    }
    if (rc != MPA_OK) return rc;
  }
#if MPA_MEASURE
  if (const char* hp = std::getenv("MPA_HOST_PROF"); hp && *hp == '1') {
    static const char* names[mpa::kHpKeys] = {"asyncmap", "flush", "pre_consume", "prearm", "launch call", "waitany",
                                              "harvest", "post", "stage_update"};
    std::fprintf(stderr, "[mpa host prof] %lld epochs, per epoch (us) / per call (us):\n", (long long)epochs);
    for (int k = 0; k < mpa::kHpKeys; ++k) {
      const int64_t ns = mpa::g_hprof.ns[k].exchange(0), cnt = mpa::g_hprof.n[k].exchange(0);
      if (cnt)
        std::fprintf(stderr, "  %-12s %8.2f / %8.2f  (%lld calls)\n", names[k], double(ns) / 1e3 / double(epochs > 0 ? epochs : 1),
                     double(ns) / 1e3 / double(cnt), (long long)cnt);
    }
  }
#endif
  if (fuse) {
    rc = guarded([&] {
      mpa::hip_set_ahead(c, 0, up.dtype, elems, w_all.data(), n, up.eta, up.x, up.mirror, up.msg_bf16);
      mpa::hip_set_defer_end(c, false);
      restore.on = false;
      mpa::hip_flush(c);  // the last call's harvests and update
    });
  }
  return rc;
}
}  // namespace
extern "C" {

int mpa_lsq_descent(mpa_pool* pool, mpa_comm* comm, int dtype, void* x, int64_t cols, void* recvbuf,
                    size_t recvbuf_bytes, void* isendbuf, size_t isendbuf_bytes, void* irecvbuf, size_t irecvbuf_bytes,
                    int nwait_kind, int64_t nwait, mpa_nwait_fn nwait_fn, void* nwait_ctx, double eta,
                    double stale_weight, int64_t epochs) {
  int rc = guarded([&] {
    if (!pool) mpa::fail(MPA_ARGUMENT_ERROR, "pool is NULL");
    if (dtype != MPA_F32 && dtype != MPA_F64) mpa::fail(MPA_ARGUMENT_ERROR, "lsq_descent: dtype must be F32 or F64");
    if (cols <= 0 || epochs < 0) mpa::fail(MPA_ARGUMENT_ERROR, "lsq_descent: bad cols / epochs");
  });
  if (rc != MPA_OK) return rc;
  const size_t es = dtype == MPA_F64 ? 8 : 4;
  return descent_loop(pool, comm, x, size_t(cols) * es, es, recvbuf, recvbuf_bytes, isendbuf, isendbuf_bytes, irecvbuf,
                      irecvbuf_bytes, nwait_kind, nwait, nwait_fn, nwait_ctx, stale_weight, epochs,
                      DescentUpdate{dtype, cols, eta, x, nullptr, false});
}

int mpa_nwait_first_plus(void* ctx, int64_t epoch, const int64_t* repochs, int64_t n) {
  if (!ctx || !repochs || n <= 0) return -1;
  const int64_t k = *static_cast<const int64_t*>(ctx);
  if (repochs[0] != epoch) return 0;
  int64_t fresh = 0;
  for (int64_t i = 1; i < n; ++i) fresh += repochs[i] == epoch;
  return fresh >= k ? 1 : 0;
}

int mpa_lsqb_update(mpa_comm* comm, void* x32, void* xb16, const void* recvbuf, int64_t nchunks, int64_t elems,
                    const double* weights, double eta) {
  if (!xb16) return guarded([&] { mpa::fail(MPA_ARGUMENT_ERROR, "lsqb_update: the bf16 iterate is NULL"); });
  return aggregate_impl(comm, MPA_F32, recvbuf, nchunks, elems, weights, x32, 1, eta, xb16);
}

int mpa_lsqb_descent(mpa_pool* pool, mpa_comm* comm, void* x32, void* xb16, int64_t elems, void* recvbuf,
                     size_t recvbuf_bytes, void* isendbuf, size_t isendbuf_bytes, void* irecvbuf,
                     size_t irecvbuf_bytes, int nwait_kind, int64_t nwait, mpa_nwait_fn nwait_fn, void* nwait_ctx,
                     double eta, double stale_weight, int64_t epochs) {
  int rc = guarded([&] {
    if (!pool) mpa::fail(MPA_ARGUMENT_ERROR, "pool is NULL");
    if (!x32 || !xb16 || elems <= 0 || epochs < 0) mpa::fail(MPA_ARGUMENT_ERROR, "lsqb_descent: bad arguments");
  });
  if (rc != MPA_OK) return rc;
  return descent_loop(pool, comm, xb16, size_t(elems) * 2, 4, recvbuf, recvbuf_bytes, isendbuf, isendbuf_bytes, irecvbuf,
                      irecvbuf_bytes, nwait_kind, nwait, nwait_fn, nwait_ctx, stale_weight, epochs,
                      DescentUpdate{MPA_F32, elems, eta, x32, xb16, true});
}

int mpa_generate(void* out, int dtype, uint64_t seed, uint32_t stream, uint64_t e0, int64_t count, double scale,
                 void* hip_stream) {
  return guarded([&] {
    if (dtype != MPA_F32 && dtype != MPA_F64 && dtype != MPA_BF16) mpa::fail(MPA_ARGUMENT_ERROR, "generate: bad dtype");
    if (count < 0 || (count > 0 && !out)) mpa::fail(MPA_ARGUMENT_ERROR, "generate: bad arguments");
    HIPCHECK_C(mpa::launch_generate(out, dtype, seed, stream, e0, count, scale, static_cast<hipStream_t>(hip_stream)));
  });
}

int mpa_read_bandwidth(const void* buf, size_t bytes, int grid, int reps, void* hip_stream, double* gbps_out) {
  return guarded([&] {
    if (!buf || bytes < 16 || (bytes & 15) || (reinterpret_cast<uintptr_t>(buf) & 15) || grid < 1 || grid > 65536 ||
        reps < 1 || !gbps_out)
      mpa::fail(MPA_ARGUMENT_ERROR, "read_bandwidth: bad arguments");
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    uint32_t* sink = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIPCHECK_C(hipMalloc(&sink, sizeof(uint32_t) * size_t(grid)));
    hipError_t e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = mpa::launch_read_peak(buf, bytes, grid, sink, s);  // warm-up
    if (e == hipSuccess) e = hipEventRecord(e0, s);
    for (int r = 0; r < reps && e == hipSuccess; ++r) e = mpa::launch_read_peak(buf, bytes, grid, sink, s);
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(sink);
    HIPCHECK_C(e);
    *gbps_out = ms > 0.f ? double(bytes) * reps / (double(ms) * 1e-3) / 1e9 : 0.0;
  });
}

}  // extern "C"
