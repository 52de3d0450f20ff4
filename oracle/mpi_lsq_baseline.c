/*
 * ORACLE / CPU BASELINE — MEASUREMENT INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
 *
 * BASELINE configs[0] as the reference runs it: a coordinator process and n worker
 * PROCESSES on host cores, over a real MPI library (MPICH, the implementation MPI.jl binds
 * by default).  Rank 0 runs the C restatement of src/MPIAsyncPools.jl's asyncmap!
 * (asyncpool_oracle.c) with the reference's own verbs (Isend + Irecv!, Test!, Waitany!,
 * Waitall!; :99,137-138,161,212) and the coordinator loop of examples/iterative_example.jl:
 * 37-47 (asyncmap!(nwait), then x -= eta * (n / #fresh) * sum of the fresh chunks); ranks
 * 1..n run its worker_main (:55-82) with the least-squares task in place of the sleep:
 * receive x, reply g_i = A_i^T (A_i x - b_i) computed in fp64 on the worker's row shard
 * (single-threaded), until the control tag (:49-52).  Data: the Philox layout of philox.h,
 * the device's own, so the shards are the bench's.
 *
 * The real reference (Julia + MPI.jl) is absent from this image: bench.py reports this
 * program as cpu_baseline.kind = "mpi" (a port of the coordinator over the same MPI).
 *
 *   mpiexec -n <n+1> mpi_lsq_baseline --rows R --cols D --nwait K --seconds S [--seed X]
 * prints one JSON line on rank 0.
 */
#define _GNU_SOURCE
#include <math.h>
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "asyncpool_oracle.h"
#include "philox.h"

enum { DATA_TAG = 0, CONTROL_TAG = 999 };

static uint64_t now_ns(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

typedef struct {
  MPI_Request* rreq;
  MPI_Request* sreq;
} mpi_ctx;

/* MPI.Isend(isendbufs[i]) + MPI.Irecv!(irecvbufs[i]) (:137-138); the send request is
 * completed at the next post to the same worker (the reference's Wait!(sreqs[i]), :113) */
static void t_isend_irecv(void* c, int64_t i, int64_t rank, const uint8_t* sbuf, size_t sl, uint8_t* rbuf, size_t rl,
                          int64_t tag) {
  mpi_ctx* m = (mpi_ctx*)c;
  MPI_Wait(&m->sreq[i], MPI_STATUS_IGNORE);
  MPI_Isend(sbuf, (int)sl, MPI_BYTE, (int)rank, (int)tag, MPI_COMM_WORLD, &m->sreq[i]);
  MPI_Irecv(rbuf, (int)rl, MPI_BYTE, (int)rank, (int)tag, MPI_COMM_WORLD, &m->rreq[i]);
}
static int t_test(void* c, int64_t i) {
  int flag = 0;
  MPI_Test(&((mpi_ctx*)c)->rreq[i], &flag, MPI_STATUS_IGNORE);
  return flag;
}
static int64_t t_waitany(void* c, int64_t n, const uint8_t* live) {
  (void)live;
  int idx = MPI_UNDEFINED;
  MPI_Waitany((int)n, ((mpi_ctx*)c)->rreq, &idx, MPI_STATUS_IGNORE);
  return idx == MPI_UNDEFINED ? -1 : idx;
}
static void t_waitall(void* c, int64_t n, const uint8_t* live) {
  (void)live;
  MPI_Waitall((int)n, ((mpi_ctx*)c)->rreq, MPI_STATUSES_IGNORE);
}
static uint64_t t_time_ns(void* c) {
  (void)c;
  return now_ns();
}

static long long arg(int argc, char** argv, const char* name, long long dflt) {
  for (int k = 1; k + 1 < argc; ++k)
    if (!strcmp(argv[k], name)) return atoll(argv[k + 1]);
  return dflt;
}

/* the worker program: examples/iterative_example.jl:55-82 with g = A^T (A x - b) */
static void worker(int rank, int64_t rows, int64_t cols, uint64_t seed) {
  const int64_t row0 = (int64_t)(rank - 1) * rows;
  double* A = malloc(sizeof(double) * (size_t)(rows * cols));
  double* b = malloc(sizeof(double) * (size_t)rows);
  const double sa = 1.0 / sqrt((double)cols);
  for (int64_t e = 0; e < rows * cols; ++e)
    A[e] = (double)orc_unit_f32(orc_philox_word(seed, 0, (uint64_t)(row0 * cols + e))) * sa;
  for (int64_t r = 0; r < rows; ++r) b[r] = (double)orc_unit_f32(orc_philox_word(seed, 1, (uint64_t)(row0 + r)));
  double* x = malloc(sizeof(double) * (size_t)cols);
  double* g = malloc(sizeof(double) * (size_t)cols);
  MPI_Barrier(MPI_COMM_WORLD);
  for (;;) {
    MPI_Status st;
    MPI_Recv(x, (int)cols, MPI_DOUBLE, 0, MPI_ANY_TAG, MPI_COMM_WORLD, &st);
    if (st.MPI_TAG == CONTROL_TAG) break;
    memset(g, 0, sizeof(double) * (size_t)cols);
    for (int64_t r = 0; r < rows; ++r) {
      const double* a = A + r * cols;
      double d = -b[r];
      for (int64_t j = 0; j < cols; ++j) d += a[j] * x[j];
      for (int64_t j = 0; j < cols; ++j) g[j] += d * a[j];
    }
    MPI_Send(g, (int)cols, MPI_DOUBLE, 0, st.MPI_TAG, MPI_COMM_WORLD);
  }
  free(A);
  free(b);
  free(x);
  free(g);
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank = 0, size = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  const int64_t n = size - 1;
  const int64_t rows_total = arg(argc, argv, "--rows", 3 << 12), cols = arg(argc, argv, "--cols", 64);
  const int64_t nwait = arg(argc, argv, "--nwait", 2);
  const double seconds = (double)arg(argc, argv, "--seconds", 10);
  const uint64_t seed = (uint64_t)arg(argc, argv, "--seed", 1234);
  if (n < 1 || rows_total % n || nwait < 0 || nwait > n) {
    if (rank == 0) fprintf(stderr, "usage: mpiexec -n <n+1> mpi_lsq_baseline --rows R --cols D --nwait K --seconds S\n");
    MPI_Abort(MPI_COMM_WORLD, 2);
  }
  const int64_t rows = rows_total / n;
  if (rank != 0) {
    worker(rank, rows, cols, seed);
    MPI_Finalize();
    return 0;
  }
  MPI_Barrier(MPI_COMM_WORLD);  /* every worker has its shard before the clock starts */
  mpi_ctx m = {malloc(sizeof(MPI_Request) * (size_t)n), malloc(sizeof(MPI_Request) * (size_t)n)};
  for (int64_t i = 0; i < n; ++i) m.rreq[i] = m.sreq[i] = MPI_REQUEST_NULL;
  orc_transport tp = {&m, t_isend_irecv, t_test, t_waitany, t_waitall, t_time_ns, NULL};
  orc_pool* p = orc_pool_create(n, NULL, 0, n);
  const size_t xb = sizeof(double) * (size_t)cols;
  double* x = calloc((size_t)cols, sizeof(double));
  uint8_t* isend = calloc((size_t)n, xb);
  double* recv = calloc((size_t)(n * cols), sizeof(double));
  double* irecv = calloc((size_t)(n * cols), sizeof(double));
  /* step size 0.9 / L, L ~ ||A||^2 (bench.py step_size) */
  const double mrows = (double)rows_total, sq = 1.0 + sqrt((double)cols / mrows);
  const double eta = 0.9 / (mrows / (3.0 * (double)cols) * sq * sq);
  const uint64_t t0 = now_ns();
  int64_t epochs = 0;
  for (;;) {
    const int rc = orc_asyncmap(p, &tp, (const uint8_t*)x, xb, (uint8_t*)recv, xb * (size_t)n, (size_t)(n * cols), isend,
                                xb * (size_t)n, (uint8_t*)irecv, xb * (size_t)n, ORC_NWAIT_INT, nwait, NULL, NULL, "Int64",
                                p->epoch + 1, DATA_TAG);
    if (rc != ORC_OK) {
      fprintf(stderr, "asyncmap! failed: %s\n", p->errmsg);
      MPI_Abort(MPI_COMM_WORLD, 3);
    }
    ++epochs;
    /* examples/iterative_example.jl:41-46: consume the fresh chunks */
    int64_t fresh = 0;
    for (int64_t i = 0; i < n; ++i) fresh += p->repochs[i] == p->epoch;
    const double w = fresh ? (double)n / (double)fresh : 0.0;
    for (int64_t i = 0; i < n; ++i)
      if (p->repochs[i] == p->epoch)
        for (int64_t j = 0; j < cols; ++j) x[j] -= eta * w * recv[i * cols + j];
    if ((double)(now_ns() - t0) * 1e-9 >= seconds) break;
  }
  const double el = (double)(now_ns() - t0) * 1e-9;
  /* drain, then the control tag (examples/iterative_example.jl:49-52) */
  orc_waitall(p, &tp, (uint8_t*)recv, xb * (size_t)n, (size_t)(n * cols), (uint8_t*)irecv, xb * (size_t)n);
  for (int64_t i = 0; i < n; ++i) MPI_Wait(&m.sreq[i], MPI_STATUS_IGNORE);
  for (int64_t r = 1; r <= n; ++r) MPI_Send(x, (int)cols, MPI_DOUBLE, (int)r, CONTROL_TAG, MPI_COMM_WORLD);
  double xn = 0;
  for (int64_t j = 0; j < cols; ++j) xn += x[j] * x[j];
  printf("{\"it_per_s\": %.4f, \"epochs\": %lld, \"seconds\": %.3f, \"processes\": %d, \"workers\": %lld, "
         "\"rows\": %lld, \"cols\": %lld, \"nwait\": %lld, \"x_norm\": %.6g}\n",
         (double)epochs / el, (long long)epochs, el, size, (long long)n, (long long)rows_total, (long long)cols,
         (long long)nwait, sqrt(xn));
  fflush(stdout);
  orc_pool_destroy(p);
  free(m.rreq);
  free(m.sreq);
  free(x);
  free(isend);
  free(recv);
  free(irecv);
  MPI_Finalize();
  return 0;
}
