/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * The oracle's asyncmap!/waitall! state machine (asyncpool_oracle.c, the restatement of
 * src/MPIAsyncPools.jl:35-224) driven over a REAL MPI library instead of the virtual-clock
 * transport: rank 0 is the coordinator, ranks 1..n run test/kmap2.jl's worker program
 * (:110-132: receive the epoch, sleep, reply Float64[rank, t, epoch]) with the sleep taken
 * from a scenario's per-(worker, task) schedule.  On schedules whose task completions are
 * >= 4 ms apart the order is physical, so the repochs / active / recvbuf trace must equal
 * the virtual-clock trace of the same scenario (tests/golden/traces.json): this pins the
 * oracle's transport model (MPI.Isend/Irecv!/Test!/Waitany!/Waitall!, :99,137-138,161,212)
 * against MPICH, the MPI implementation MPI.jl binds by default.  tests/test_mpi_replay.py
 * builds it (oracle/Makefile target `mpi`) where MPICH is present and runs it with mpiexec.
 *
 * Scenario file (text):  n ncols nops
 *                        n lines of ncols task durations (ns)
 *                        nops lines: "A <nwait> <send>" | "F <k> <send>" (first_plus_k)
 *                                    | "C <k> <send>" (count_k) | "W" (waitall!)
 * Output, one line per op:  repochs... | active... | recv...
 * argv[2] (optional): a factor every duration is multiplied by.  Completion order on the
 * virtual clock depends only on sums of durations along causal chains, so a uniform scale
 * keeps the trace and widens the gaps against timer and scheduling noise.
 */
#define _GNU_SOURCE
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "asyncpool_oracle.h"

enum { CONTROL_TAG = 999 };

typedef struct {
  int64_t n;
  MPI_Request* rreq;
} mpi_ctx;

static void t_isend_irecv(void* c, int64_t i, int64_t rank, const uint8_t* sbuf, size_t sl, uint8_t* rbuf, size_t rl,
                          int64_t tag) {
  mpi_ctx* m = (mpi_ctx*)c;
  /* the messages are 8 bytes: MPI_Send completes eagerly, as the reference's Isend + later
   * Wait! does (:137, :113) */
  MPI_Send(sbuf, (int)sl, MPI_BYTE, (int)rank, (int)tag, MPI_COMM_WORLD);
  MPI_Irecv(rbuf, (int)rl, MPI_BYTE, (int)rank, (int)tag, MPI_COMM_WORLD, &m->rreq[i]);
}
static int t_test(void* c, int64_t i) {
  mpi_ctx* m = (mpi_ctx*)c;
  int flag = 0;
  MPI_Test(&m->rreq[i], &flag, MPI_STATUS_IGNORE);
  return flag;
}
static int64_t t_waitany(void* c, int64_t n, const uint8_t* live) {
  mpi_ctx* m = (mpi_ctx*)c;
  (void)live; /* completed requests are MPI_REQUEST_NULL already */
  int idx = MPI_UNDEFINED;
  MPI_Waitany((int)n, m->rreq, &idx, MPI_STATUS_IGNORE);
  return idx == MPI_UNDEFINED ? -1 : idx;
}
static void t_waitall(void* c, int64_t n, const uint8_t* live) {
  mpi_ctx* m = (mpi_ctx*)c;
  (void)live;
  MPI_Waitall((int)n, m->rreq, MPI_STATUSES_IGNORE);
}
static uint64_t t_time_ns(void* c) {
  (void)c;
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static int pred_first_plus(void* ctx, int64_t epoch, const int64_t* repochs, int64_t n) {
  const int64_t k = *(const int64_t*)ctx;
  if (repochs[0] != epoch) return 0;
  int64_t f = 0;
  for (int64_t i = 1; i < n; ++i) f += repochs[i] == epoch;
  return f >= k;
}
static int pred_count(void* ctx, int64_t epoch, const int64_t* repochs, int64_t n) {
  const int64_t k = *(const int64_t*)ctx;
  int64_t f = 0;
  for (int64_t i = 0; i < n; ++i) f += repochs[i] == epoch;
  return f >= k;
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank = 0, size = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  FILE* f = argc > 1 ? fopen(argv[1], "r") : NULL;
  long long n = 0, ncols = 0, nops = 0;
  if (!f || fscanf(f, "%lld %lld %lld", &n, &ncols, &nops) != 3 || n != size - 1) {
    if (rank == 0) fprintf(stderr, "usage: mpiexec -n <n+1> mpi_replay <scenario>\n");
    MPI_Abort(MPI_COMM_WORLD, 2);
  }
  const long long scale = argc > 2 ? atoll(argv[2]) : 1;
  int64_t* dur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n * ncols));
  for (long long k = 0; k < n * ncols; ++k) {
    long long v = 0;
    if (fscanf(f, "%lld", &v) != 1) MPI_Abort(MPI_COMM_WORLD, 2);
    dur[k] = v * (scale > 0 ? scale : 1);
  }

  MPI_Barrier(MPI_COMM_WORLD);  /* every worker is up before the first post */
  if (rank != 0) {
    /* test/kmap2.jl:76-99: the worker's t-th task sleeps, then replies [rank, t, epoch] */
    fclose(f);
    for (int64_t t = 1;; ++t) {
      MPI_Status st;
      double epoch = 0;
      /* poll with short sleeps instead of MPICH's spinning receive: n + 1 spinning ranks on
       * fewer cores delayed the sleepers' wake-ups by milliseconds */
      MPI_Request rq;
      MPI_Irecv(&epoch, 1, MPI_DOUBLE, 0, MPI_ANY_TAG, MPI_COMM_WORLD, &rq);
      for (int done = 0;;) {
        MPI_Test(&rq, &done, &st);
        if (done) break;
        const struct timespec nap = {0, 20000};
        nanosleep(&nap, NULL);
      }
      if (st.MPI_TAG == CONTROL_TAG) break;
      const int64_t d = dur[(rank - 1) * ncols + (t - 1) % ncols];
      struct timespec ts = {(time_t)(d / 1000000000), (long)(d % 1000000000)};
      nanosleep(&ts, NULL);
      double reply[3] = {(double)rank, (double)t, epoch};
      MPI_Send(reply, 3, MPI_DOUBLE, 0, st.MPI_TAG, MPI_COMM_WORLD);
    }
    free(dur);
    MPI_Finalize();
    return 0;
  }

  mpi_ctx m = {n, (MPI_Request*)malloc(sizeof(MPI_Request) * (size_t)n)};
  for (long long i = 0; i < n; ++i) m.rreq[i] = MPI_REQUEST_NULL;
  orc_transport tp = {&m, t_isend_irecv, t_test, t_waitany, t_waitall, t_time_ns, NULL};
  orc_pool* p = orc_pool_create(n, NULL, 0, n);
  double send = 0, *isend = calloc((size_t)n, sizeof(double));
  double *recv = calloc((size_t)(3 * n), sizeof(double)), *irecv = calloc((size_t)(3 * n), sizeof(double));
  for (long long op = 0; op < nops; ++op) {
    char kind[4] = {0};
    long long a1 = 0, a2 = 0;
    if (fscanf(f, "%3s", kind) != 1) MPI_Abort(MPI_COMM_WORLD, 2);
    int rc;
    if (kind[0] == 'W') {
      rc = orc_waitall(p, &tp, (uint8_t*)recv, sizeof(double) * 3 * n, 3 * n, (uint8_t*)irecv, sizeof(double) * 3 * n);
    } else {
      if (fscanf(f, "%lld %lld", &a1, &a2) != 2) MPI_Abort(MPI_COMM_WORLD, 2);
      send = (double)a2;
      int64_t k = a1;
      const int fn = kind[0] != 'A';
      rc = orc_asyncmap(p, &tp, (const uint8_t*)&send, sizeof(double), (uint8_t*)recv, sizeof(double) * 3 * n, 3 * n,
                        (uint8_t*)isend, sizeof(double) * n, (uint8_t*)irecv, sizeof(double) * 3 * n,
                        fn ? ORC_NWAIT_FN : ORC_NWAIT_INT, fn ? 0 : k,
                        kind[0] == 'F' ? pred_first_plus : kind[0] == 'C' ? pred_count : NULL, &k, "Int64",
                        p->epoch + 1, 0);
    }
    if (rc != ORC_OK) {
      fprintf(stderr, "op %lld failed: %s\n", op, p->errmsg);
      MPI_Abort(MPI_COMM_WORLD, 3);
    }
    for (long long i = 0; i < n; ++i) printf("%lld ", (long long)p->repochs[i]);
    printf("|");
    for (long long i = 0; i < n; ++i) printf(" %d", (int)p->active[i]);
    printf(" |");
    for (long long i = 0; i < 3 * n; ++i) printf(" %.17g", recv[i]);
    printf("\n");
  }
  fclose(f);
  /* drain what is still outstanding, then the control tag (examples/iterative_example.jl:49-52) */
  orc_waitall(p, &tp, (uint8_t*)recv, sizeof(double) * 3 * n, 3 * n, (uint8_t*)irecv, sizeof(double) * 3 * n);
  for (long long r = 1; r <= n; ++r) {
    double z = 0;
    MPI_Send(&z, 1, MPI_DOUBLE, (int)r, CONTROL_TAG, MPI_COMM_WORLD);
  }
  fflush(stdout);
  orc_pool_destroy(p);
  free(m.rreq);
  free(isend);
  free(recv);
  free(irecv);
  free(dur);
  MPI_Finalize();
  return 0;
}
