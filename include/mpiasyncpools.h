/*
 * mpiasyncpools.h — C ABI of the MI355X-native `asyncmap!` hot path of MPIAsyncPools.jl
 * (severinson/MPIStragglers.jl, package `MPIAsyncPools` v0.1.0).
 *
 * Plain C: opaque handles, raw pointers, byte sizes, int status codes.  No torch or HIP
 * types appear in any signature (streams are passed as `void*` = hipStream_t).
 *
 * Reference interface each entry point replaces (file:line in the reference tree):
 *
 *   mpa_pool_create / mpa_pool_destroy
 *       MPIAsyncPool(ranks; epoch0, nwait)            src/MPIAsyncPools.jl:35-43
 *       MPIAsyncPool(n)                               src/MPIAsyncPools.jl:46
 *   mpa_pool_ranks / _sepochs / _repochs / _active / _stimestamps / _latency /
 *   mpa_pool_nwait / mpa_pool_epoch   (borrowed, aliasing the pool's state)
 *       the MPIAsyncPool fields                       src/MPIAsyncPools.jl:25-34
 *   mpa_asyncmap
 *       Base.asyncmap!(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm;
 *                      nwait, epoch, tag) -> repochs  src/MPIAsyncPools.jl:68-188
 *   mpa_waitall
 *       waitall!(pool, recvbuf, irecvbuf) -> repochs  src/MPIAsyncPools.jl:195-224
 *   mpa_comm_*
 *       the `comm::MPI.Comm` argument (MPI.COMM_WORLD, examples/iterative_example.jl:8)
 *       together with the worker programs that answer on it (worker_main,
 *       examples/iterative_example.jl:55-82, test/kmap1.jl:23-33,
 *       test/kmap2.jl:76-99): a communicator whose ranks 1..n are device workers,
 *       each running a registered task on its own HIP stream.
 *   mpa_comm_shutdown
 *       the control-tag shutdown (examples/iterative_example.jl:49-52,
 *       test/kmap2.jl:14-18)
 *   mpa_aggregate / mpa_lsq_update
 *       the coordinator's consumption of `recvbuf` chunks
 *       (examples/iterative_example.jl:41-46, test/kmap2.jl:37-51) as device kernels.
 *
 * Status codes map onto the reference's exceptions: MPA_ARGUMENT_ERROR -> ArgumentError,
 * MPA_DIMENSION_MISMATCH -> DimensionMismatch, MPA_ERROR -> ErrorException; the message
 * (same text as the reference's) is returned by mpa_last_error() on the calling thread.
 *
 * Buffers.  With the HIP transport, sendbuf/recvbuf/isendbuf/irecvbuf are device
 * pointers on the coordinator's GPU; all device work the pool enqueues for the
 * coordinator (harvest copies into recvbuf, copies of sendbuf into isendbuf) is ordered
 * on the comm's coordinator stream (mpa_comm_set_stream), so a caller that reads recvbuf
 * or writes sendbuf on that stream needs no further synchronisation.  With the SIM
 * transport (host-logic tests only) they are host pointers.
 *
 * Threading: one coordinator thread per pool, as in the reference.  The nwait callback
 * runs synchronously on the calling thread.  Not re-entrant per pool.
 */
#ifndef MPIASYNCPOOLS_H
#define MPIASYNCPOOLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPA_ABI_VERSION 3

typedef struct mpa_pool mpa_pool;
typedef struct mpa_comm mpa_comm;

enum mpa_status {
  MPA_OK = 0,
  MPA_ARGUMENT_ERROR = 1,     /* ArgumentError      (src/MPIAsyncPools.jl:71,73,74,197) */
  MPA_DIMENSION_MISMATCH = 2, /* DimensionMismatch  (src/MPIAsyncPools.jl:75-77,198,199) */
  MPA_ERROR = 3,              /* ErrorException     (src/MPIAsyncPools.jl:157) */
  MPA_DEVICE_ERROR = 4,       /* a HIP call or a device-side check failed */
  MPA_CALLBACK_ERROR = 5,     /* the nwait callback reported an exception */
};

enum mpa_dtype { MPA_F32 = 0, MPA_F64 = 1, MPA_BF16 = 2 };

enum mpa_transport {
  MPA_TRANSPORT_HIP = 0, /* the product: device workers on HIP streams */
  MPA_TRANSPORT_SIM = 1, /* deterministic virtual-clock host transport, for host-logic tests */
  MPA_TRANSPORT_HOST = 2, /* multi-process mailbox protocol with host-executed test workers,
                             for tests of the N > 1 control plane without a GPU */
  MPA_TRANSPORT_MPI = 3,  /* a real MPI communicator whose ranks run arbitrary worker
                             programs (libmpiasyncpools_mpi.so, mpiasyncpools_mpi.h) */
};

enum mpa_nwait_kind { MPA_NWAIT_INT = 0, MPA_NWAIT_FN = 1, MPA_NWAIT_OTHER = 2 };

enum mpa_task {
  MPA_TASK_NONE = 0,
  MPA_TASK_ECHO = 1,       /* reply = the received bytes (zero padded / truncated) */
  MPA_TASK_KMAP1 = 2,      /* reply = Float64(rank)            (test/kmap1.jl:24-32) */
  MPA_TASK_KMAP2 = 3,      /* reply = Float64[rank, t, epoch]  (test/kmap2.jl:76-99) */
  MPA_TASK_LSQ = 4,        /* reply = A_i^T (A_i x - b_i)      (BASELINE workload) */
  MPA_TASK_LSQ_BATCH = 5,  /* reply = A_i^T (A_i X - B_i), X cols x k (bf16 MFMA) */
};

/* observation points of the state machine, the step kinds of a gated replay
 * (mpa_comm_set_gate): before phase 1 of asyncmap! (src/MPIAsyncPools.jl:91), before each
 * MPI.Waitany! with a live request (:161), before MPI.Waitall! (:212) */
enum mpa_gate_step { MPA_GATE_CALL = 0, MPA_GATE_WAIT = 1, MPA_GATE_WAITALL = 2 };

/* nwait::Function — nwait(epoch, repochs)::Bool (src/MPIAsyncPools.jl:153).
 * Return 1 (true), 0 (false) or a negative value if the callback raised. */
typedef int (*mpa_nwait_fn)(void* ctx, int64_t epoch, const int64_t* repochs, int64_t n);

/* A ready-made native nwait predicate (BASELINE configs[3]): true when worker 1 is fresh
 * (repochs[0] == epoch, the predicate of test/kmap2.jl:65) and at least *(int64_t*)ctx of
 * the other workers are fresh too. */
int mpa_nwait_first_plus(void* ctx, int64_t epoch, const int64_t* repochs, int64_t n);

int mpa_abi_version(void);
const char* mpa_last_error(void);
/* build description: target arch and the least-squares kernel variant in use */
const char* mpa_build_info(void);
/* tuning knobs for measurement: "lsq_variant" (index of the compiled fp32 1024-column
 * kernel variants, DESIGN.md §Kernel tuning), "lsq_grid" (workgroups per least-squares
 * task for tasks registered afterwards; 0 = default) */
int mpa_tune(const char* key, int64_t value);

/* ---- pool: src/MPIAsyncPools.jl:24-46 -------------------------------------------- */
/* ranks == NULL means ranks 1:n (src/MPIAsyncPools.jl:46). */
int mpa_pool_create(int64_t n, const int64_t* ranks, int64_t epoch0, int64_t nwait, mpa_pool** out);
void mpa_pool_destroy(mpa_pool* pool);
int64_t mpa_pool_size(const mpa_pool* pool);
int64_t* mpa_pool_ranks(mpa_pool* pool);
int64_t* mpa_pool_sepochs(mpa_pool* pool);
int64_t* mpa_pool_repochs(mpa_pool* pool);
uint8_t* mpa_pool_active(mpa_pool* pool);
int64_t* mpa_pool_stimestamps(mpa_pool* pool);
double* mpa_pool_latency(mpa_pool* pool);
int64_t* mpa_pool_nwait(mpa_pool* pool);
int64_t* mpa_pool_epoch(mpa_pool* pool);

/* ---- asyncmap! / waitall!: src/MPIAsyncPools.jl:68-188, 195-224 ------------------- */
/* recvbuf_length is the element count of recvbuf (the reference checks
 * `mod(length(recvbuf), n) == 0`, src/MPIAsyncPools.jl:77).  On success *repochs_out
 * (if non-NULL) receives mpa_pool_repochs(pool): the same aliased vector the reference
 * returns (src/MPIAsyncPools.jl:187). */
int mpa_asyncmap(mpa_pool* pool,
                 const void* sendbuf, size_t sendbuf_bytes,
                 void* recvbuf, size_t recvbuf_bytes, size_t recvbuf_length,
                 void* isendbuf, size_t isendbuf_bytes,
                 void* irecvbuf, size_t irecvbuf_bytes,
                 mpa_comm* comm,
                 int nwait_kind, int64_t nwait, mpa_nwait_fn nwait_fn, void* nwait_ctx,
                 const char* nwait_typename,
                 int64_t epoch, int64_t tag,
                 int64_t** repochs_out);

int mpa_waitall(mpa_pool* pool,
                void* recvbuf, size_t recvbuf_bytes, size_t recvbuf_length,
                void* irecvbuf, size_t irecvbuf_bytes,
                int64_t** repochs_out);

/* ---- comm: MPI.Comm + the worker programs ------------------------------------------ */
/* nworkers device workers with ranks 1..nworkers (rank 0 is the coordinator), all on the
 * calling thread's current HIP device.  devices[w] (w = rank-1) may be given to assert
 * that: a process serves the workers of its own device only, so any other entry is an
 * ArgumentError; workers of other GPUs are served by their own processes
 * (mpa_comm_create_dist, one process per GPU).  NULL = the current device. */
int mpa_comm_create(int transport, int64_t nworkers, const int* devices, mpa_comm** out);
void mpa_comm_destroy(mpa_comm* comm);
int64_t mpa_comm_size(const mpa_comm* comm); /* nworkers + 1, as MPI.Comm_size */
/* coordinator stream (hipStream_t).  NULL (the legacy default stream) selects the comm's own
 * coordinator stream: a blocking stream, so HIP orders it with the caller's NULL-stream work
 * both ways, while the comm's epoch steps and harvests no longer wait, as every NULL-stream
 * command does, for the stragglers' tasks running on the worker streams (MPA_OWN_COORD=0:
 * the NULL stream itself). */
int mpa_comm_set_stream(mpa_comm* comm, void* stream);
/* worker tasks (rank in 1..nworkers) */
int mpa_comm_set_task_kmap(mpa_comm* comm, int64_t rank, int task /* ECHO/KMAP1/KMAP2 */);
/* A_i: rows x cols row-major with leading dimension lda (elements, lda % (16/sizeof) == 0),
 * b_i: rows, both device pointers on the worker's device; x = cols elements and the reply
 * g_i = cols elements, dtype MPA_F32 or MPA_F64. */
int mpa_comm_set_task_lsq(mpa_comm* comm, int64_t rank, int dtype, int64_t rows, int64_t cols,
                          const void* A, int64_t lda, const void* b);
/* the batched multi-iterate variant (BASELINE configs[4]): G_i = A_i^T (A_i X - B_i) with
 * A_i rows x cols bf16 (leading dimension lda, lda % 8 == 0, 16-byte aligned), B_i rows x k
 * bf16 (row-major), the message X = cols x k bf16 and the reply G_i = cols x k fp32, both
 * row-major; k == 64, cols % 32 == 0, cols <= 4096.  bf16 MFMA with fp32 accumulation. */
int mpa_comm_set_task_lsq_batch(mpa_comm* comm, int64_t rank, int64_t rows, int64_t cols, int64_t k,
                                const void* A, int64_t lda, const void* B);
/* straggler emulation: task t (1-based) of the worker is delayed by
 * delays_ns[(t-1) % count] before it computes; count == 0 clears the schedule */
int mpa_comm_set_delays(mpa_comm* comm, int64_t rank, const int64_t* delays_ns, int64_t count);
/* tasks completed (replies published) by a worker so far */
int64_t mpa_comm_tasks_done(mpa_comm* comm, int64_t rank);
/* control channel: wait for every outstanding task, then refuse further posts */
int mpa_comm_shutdown(mpa_comm* comm);
/* gated replay (a test mode; HIP and HOST transports, rank 0): fixes the order in which
 * completions become visible to MPI.Test! / Waitany! / Waitall! (src/MPIAsyncPools.jl:99,
 * 161,212).  Step k (kinds[k] = MPA_GATE_*) is taken at the k-th observation point of the
 * state machine and releases one more completion of each worker rank in
 * ranks[offsets[k] .. offsets[k+1]); a request reads as complete once its task has
 * finished and been released, and the step waits until every task it releases has
 * finished.  A step of the wrong kind is an error; after the last step the next
 * observation switches the gate off; nsteps == 0 switches it off now.  Schedules come from
 * the oracle's virtual clock (oracle/oracle.py gate_schedule), so the device replays the
 * oracle's trace bit for bit whatever the physical completion order. */
int mpa_comm_set_gate(mpa_comm* comm, int64_t nsteps, const int* kinds, const int64_t* offsets,
                      const int64_t* ranks);
/* event counters (tests, diagnostics); -1 for a name the transport does not count.  HIP
 * rank 0: "held" stale re-dispatches whose launch was held (src/MPIAsyncPools.jl:177-184,
 * DESIGN.md §5), "held_joined" of them launched inside a later batch, "held_alone" launched
 * on their own (a wait that would block, a gated release, waitall!, shutdown);
 * "gate_steps" gated-replay steps taken; "head_steps" / "epoch_kernels" native-loop epoch
 * steps run at the head of a task launch / as their own kernel, "prearmed" /
 * "prearm_cancelled" pre-armed launches released / cancelled, "prearm_same" pre-armed
 * launches released with the step they predicted (no mailbox read), "stale_deferred" held
 * re-dispatches whose copies joined the next epoch step, "task_launches"
 * least-squares task launches, "armed" (worker process) tasks launched device-armed,
 * "sleeps" delayed tasks that slept on the device (behind a deadline kernel, or in a worker
 * process's doorbell wait), "clock_samples" host <-> device clock samples behind the deadlines,
 * "timer_late" delayed launches the host timer issued more than 1 ms after they were due,
 * "queues" CU-masked streams (HSA queues) the process holds on the comm's device,
 * "queues_past_cap" queues created past the cap (a stream kind that had none),
 * "shared_worker_streams" workers whose stream is shared past the queue cap, "reserved_cus"
 * CUs this process's task streams leave to the coordinator (MPA_RESERVE_CUS=1). */
int64_t mpa_comm_counter(mpa_comm* comm, const char* name);
/* ---- multi-process communicators: one process per GPU ------- */
/* placement[w] = the process rank that serves worker w+1 (rank 0 is the coordinator's own
 * process).  my_rank 0 creates the shared-memory mailboxes `shm_name` (POSIX shm name,
 * messages of at most max_msg_bytes each way), every other rank attaches to them after
 * rank 0 has created them.  On rank 0 the comm is used with mpa_asyncmap/mpa_waitall; on
 * the other ranks, after registering the tasks of their workers, with mpa_comm_serve.
 * transport: MPA_TRANSPORT_HIP (the product) or MPA_TRANSPORT_HOST (protocol tests). */
int mpa_comm_create_dist(int transport, int64_t nworkers, const int* placement, int my_rank,
                         const char* shm_name, size_t max_msg_bytes, mpa_comm** out);
/* worker processes: run the tasks posted to the workers placed on this rank (the
 * reference's worker_main loop, examples/iterative_example.jl:55-82) until rank 0 pauses
 * the servers or shuts the comm down */
int mpa_comm_serve(mpa_comm* comm);
/* rank 0: make every running mpa_comm_serve return (e.g. around a barrier) */
int mpa_comm_pause_servers(mpa_comm* comm);
/* rank 0 of a HIP multi-process communicator: the payload path of worker `rank` once its
 * first message was posted: 0 not yet decided / not a remote worker, 1 host shared-memory
 * mailbox, 2 device memory over xGMI (HIP IPC; MPA_XGMI=0 forces 1) */
int mpa_comm_payload_path(mpa_comm* comm, int64_t rank);
/* HIP transport: time every worker-task kernel launch with HIP events on the stream it
 * runs on (enable = 1 / 0; enable = k > 1 samples one in every k launches, and one in every
 * k epoch kernels, keeping the events' own host cost off the latency-bound critical path).
 * mpa_comm_timing returns, since its previous call:
 * out[0] launches, out[1] summed kernel milliseconds, out[2] summed algorithmic bytes
 * (A_i + b_i + x + g_i of every task in the launch), out[3] the
 * milliseconds during which at least one of those launches ran (their union: launches of
 * delayed workers run concurrently). */
int mpa_comm_set_timing(mpa_comm* comm, int enable);
int mpa_comm_timing(mpa_comm* comm, double out[4]);
/* The coordinator's epoch kernels (fused harvest + update + dispatch, the native descent
 * loop) timed under the same switch: out = {launches, total ms, bytes moved to / from
 * workers of OTHER processes (messages into their device slots over xGMI, replies from
 * their inboxes)} since the previous call.  The broadcast of the iterate
 * (src/MPIAsyncPools.jl:130-138's Isend to every idle worker) is this kernel's remote part. */
int mpa_comm_exchange_timing(mpa_comm* comm, double out[3]);
/* HIP transport, diagnostics: the task trace.  mpa_comm_set_trace(comm, capacity) starts a
 * trace of the next `capacity` posted tasks (0: off; the previous trace is dropped).
 * mpa_comm_trace copies min(count recorded, capacity) entries of 11 int64 each into `out`:
 * {rank, seq, post, due, call, ret, start, pub, gate, seen, harvest}, host steady-clock ns, 0 where
 * the task did not reach that point: post = dispatch (src/MPIAsyncPools.jl:130-137), due =
 * post + its injected delay (the reference worker's reply time), call / ret = the launch call
 * of its kernel entered / returned (the timer thread's for a delayed task), start / pub = the
 * kernel's first instruction and its completion store on the device clock (s_memrealtime,
 * mapped to host time by clock calibrations; the reference's worker programs only), gate / seen = a
 * gated replay's step that waited for it began / observed the completion, harvest = phase 1 or
 * the wait loop took it
 * (:99-104, :161-167).  A late harvest splits into launch call, queue, kernel, visibility. */
int mpa_comm_set_trace(mpa_comm* comm, int64_t capacity);
int mpa_comm_trace(mpa_comm* comm, int64_t* out, int64_t capacity, int64_t* count);
/* SIM transport only: compute time per task and the virtual clock */
int mpa_comm_sim_set_compute(mpa_comm* comm, int64_t compute_ns);
int mpa_comm_sim_advance(mpa_comm* comm, int64_t dt_ns);
int64_t mpa_comm_sim_now(const mpa_comm* comm);

/* ---- coordinator-side device kernels (HIP transport; on the coordinator stream) ---- */
/* out[c] = sum_{i=0}^{nchunks-1} weights[i] * chunk_i[c]  (fixed order, deterministic) */
int mpa_aggregate(mpa_comm* comm, int dtype, const void* recvbuf, int64_t nchunks,
                  int64_t chunk_elems, const double* weights, void* out);
/* x[c] -= eta * sum_i weights[i] * chunk_i[c]   (the iterate update of the LSQ example) */
int mpa_lsq_update(mpa_comm* comm, int dtype, void* x, const void* recvbuf, int64_t nchunks,
                   int64_t cols, const double* weights, double eta);

/* The coordinator loop of the least-squares example in native code (the structure of
 * examples/iterative_example.jl:37-47 with the BASELINE workload): `epochs` iterations of
 *     repochs = asyncmap!(pool, x, recvbuf, isendbuf, irecvbuf, comm; nwait)
 *     w_i = 1 (repochs[i] == epoch), stale_weight (older result), 0 (none yet)
 *     x  -= eta * n / sum(w) * sum_i w_i * g_i                      (mpa_lsq_update)
 * Each iteration makes exactly the calls a caller's loop makes (mpa_asyncmap, then
 * mpa_lsq_update), without an interpreter between them.  x holds cols elements; recvbuf,
 * isendbuf and irecvbuf hold n * cols, and their byte sizes are checked as asyncmap!
 * checks them (src/MPIAsyncPools.jl:75-77: DimensionMismatch) before anything is posted.
 * "Received" in the weights means a reply of the worker has been harvested at least once
 * (a worker never heard from contributes nothing, whatever the pool's epoch0). */
int mpa_lsq_descent(mpa_pool* pool, mpa_comm* comm, int dtype, void* x, int64_t cols,
                    void* recvbuf, size_t recvbuf_bytes, void* isendbuf, size_t isendbuf_bytes,
                    void* irecvbuf, size_t irecvbuf_bytes, int nwait_kind, int64_t nwait, mpa_nwait_fn nwait_fn,
                    void* nwait_ctx, double eta, double stale_weight, int64_t epochs);

/* The batched multi-iterate variant (mpa_comm_set_task_lsq_batch): the iterate X (cols x 64)
 * is kept as an fp32 master x32 and sent as its bf16 rounding xb16 (the message);
 *     x32 -= eta * sum_i weights[i] * G_i ;  xb16 = bf16(x32)        (one device kernel)
 * elems = cols * 64; recvbuf holds nchunks fp32 chunks of elems. */
int mpa_lsqb_update(mpa_comm* comm, void* x32, void* xb16, const void* recvbuf, int64_t nchunks, int64_t elems,
                    const double* weights, double eta);
/* mpa_lsq_descent for the batched variant: sendbuf = xb16 (elems bf16), recvbuf /
 * irecvbuf n * elems fp32, isendbuf n * elems bf16, update by mpa_lsqb_update. */
int mpa_lsqb_descent(mpa_pool* pool, mpa_comm* comm, void* x32, void* xb16, int64_t elems,
                     void* recvbuf, size_t recvbuf_bytes, void* isendbuf, size_t isendbuf_bytes,
                     void* irecvbuf, size_t irecvbuf_bytes, int nwait_kind, int64_t nwait, mpa_nwait_fn nwait_fn,
                     void* nwait_ctx, double eta, double stale_weight, int64_t epochs);

/* ---- synthetic data (device): Philox4x32-10 layout of DESIGN.md §Data ------------- */
/* out[k] = unit(philox(seed, stream, e0 + k)) * scale, k < count, dtype F32/F64/BF16 */
int mpa_generate(void* out, int dtype, uint64_t seed, uint32_t stream, uint64_t e0, int64_t count,
                 double scale, void* hip_stream);

/* ---- measurement: the HBM read ceiling the roofline is read against ---------------- */
/* Streams `bytes` (multiple of 16, 16-B aligned device buffer) `reps` times with a plain
 * non-temporal read kernel of `grid` 256-thread workgroups on `hip_stream` (after one
 * untimed pass) and returns the rate in GB/s (no reference counterpart: bench.py context
 * for the shard kernels' roofline fraction, SURVEY.md §8d "measured copy-kernel peak"). */
int mpa_read_bandwidth(const void* buf, size_t bytes, int grid, int reps, void* hip_stream, double* gbps_out);

#ifdef __cplusplus
}
#endif
#endif /* MPIASYNCPOOLS_H */
