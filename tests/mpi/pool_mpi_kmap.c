/*
 * TEST DRIVER for the MPI transport (libmpiasyncpools_mpi.so): the PRODUCT pool
 * (mpa_pool_create / mpa_asyncmap / mpa_waitall of libmpiasyncpools.so) on rank 0 of an
 * MPI job whose ranks 1..n run test/kmap2.jl's worker program (:110-132: receive the
 * epoch, sleep, reply Float64[rank, t, epoch]) with the sleep taken from a scenario's
 * per-(worker, task) schedule.  Scenario format and output (one line per op:
 * repochs | active | recvbuf) are those of the golden traces (tests/golden/traces.json,
 * see tests/test_mpi_transport.py); on schedules whose completions are >= 4 ms apart the
 * order is physical, so the trace must equal the virtual-clock golden trace.
 *
 * Scenario:  n ncols nops / n lines of ncols durations (ns) /
 *            nops lines "A <nwait> <send>" | "F <k> <send>" | "C <k> <send>" | "W"
 * argv[2]: a factor every duration is multiplied by (order depends only on sums).
 */
#define _GNU_SOURCE
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mpiasyncpools_mpi.h"

enum { CONTROL_TAG = 999 };

static int pred_count(void* ctx, int64_t epoch, const int64_t* repochs, int64_t n) {
  const int64_t k = *(const int64_t*)ctx;
  int64_t f = 0;
  for (int64_t i = 0; i < n; ++i) f += repochs[i] == epoch;
  return f >= k;
}

static void worker(int rank, const int64_t* dur, long long ncols) {
  for (int64_t t = 1;; ++t) {
    MPI_Status st;
    double epoch = 0;
    MPI_Request rq;
    MPI_Irecv(&epoch, 1, MPI_DOUBLE, 0, MPI_ANY_TAG, MPI_COMM_WORLD, &rq);
    for (int done = 0;;) { /* napping poll: n + 1 spinning ranks on fewer cores skew sleeps */
      MPI_Test(&rq, &done, &st);
      if (done) break;
      const struct timespec nap = {0, 20000};
      nanosleep(&nap, NULL);
    }
    if (st.MPI_TAG == CONTROL_TAG) return;
    const int64_t d = dur[(rank - 1) * ncols + (t - 1) % ncols];
    struct timespec ts = {(time_t)(d / 1000000000), (long)(d % 1000000000)};
    nanosleep(&ts, NULL);
    double reply[3] = {(double)rank, (double)t, epoch};
    MPI_Send(reply, 3, MPI_DOUBLE, 0, st.MPI_TAG, MPI_COMM_WORLD);
  }
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank = 0, size = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  FILE* f = argc > 1 ? fopen(argv[1], "r") : NULL;
  long long n = 0, ncols = 0, nops = 0;
  if (!f || fscanf(f, "%lld %lld %lld", &n, &ncols, &nops) != 3 || n != size - 1) {
    if (rank == 0) fprintf(stderr, "usage: mpiexec -n <n+1> pool_mpi_kmap <scenario> [scale]\n");
    MPI_Abort(MPI_COMM_WORLD, 2);
  }
  const long long scale = argc > 2 ? atoll(argv[2]) : 1;
  int64_t* dur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n * ncols));
  for (long long k = 0; k < n * ncols; ++k) {
    long long v = 0;
    if (fscanf(f, "%lld", &v) != 1) MPI_Abort(MPI_COMM_WORLD, 2);
    dur[k] = v * (scale > 0 ? scale : 1);
  }
  MPI_Barrier(MPI_COMM_WORLD);
  if (rank != 0) {
    fclose(f);
    worker(rank, dur, ncols);
    free(dur);
    MPI_Finalize();
    return 0;
  }

  mpa_pool* pool = NULL;
  mpa_comm* comm = NULL;
  if (mpa_pool_create(n, NULL, 0, n, &pool) != MPA_OK ||
      mpa_comm_create_mpi((int64_t)MPI_Comm_c2f(MPI_COMM_WORLD), &comm) != MPA_OK) {
    fprintf(stderr, "setup failed: %s\n", mpa_last_error());
    MPI_Abort(MPI_COMM_WORLD, 3);
  }
  /* the reference's argument checks come back as status codes with its message */
  {
    double s = 0, b[64] = {0};
    if (mpa_asyncmap(pool, &s, 8, b, 24 * n, 3 * n, b, 8 * n, b, 24 * n, comm, MPA_NWAIT_INT, n + 1, NULL, NULL,
                     "Int64", 1, 0, NULL) != MPA_ARGUMENT_ERROR ||
        !strstr(mpa_last_error(), "nwait must be in the range")) {
      fprintf(stderr, "nwait range check missing\n");
      MPI_Abort(MPI_COMM_WORLD, 4);
    }
  }
  int64_t* const repochs = mpa_pool_repochs(pool);
  const uint8_t* const active = mpa_pool_active(pool);
  double send = 0, *isend = calloc((size_t)n, sizeof(double));
  double *recv = calloc((size_t)(3 * n), sizeof(double)), *irecv = calloc((size_t)(3 * n), sizeof(double));
  const size_t rb = sizeof(double) * 3 * (size_t)n;
  for (long long op = 0; op < nops; ++op) {
    char kind[4] = {0};
    long long a1 = 0, a2 = 0;
    if (fscanf(f, "%3s", kind) != 1) MPI_Abort(MPI_COMM_WORLD, 2);
    int rc;
    int64_t* ret = NULL;
    if (kind[0] == 'W') {
      rc = mpa_waitall(pool, recv, rb, 3 * n, irecv, rb, &ret);
    } else {
      if (fscanf(f, "%lld %lld", &a1, &a2) != 2) MPI_Abort(MPI_COMM_WORLD, 2);
      send = (double)a2;
      int64_t k = a1;
      const int fn = kind[0] != 'A';
      rc = mpa_asyncmap(pool, &send, sizeof(double), recv, rb, 3 * n, isend, sizeof(double) * n, irecv, rb, comm,
                        fn ? MPA_NWAIT_FN : MPA_NWAIT_INT, fn ? 0 : k,
                        kind[0] == 'F' ? mpa_nwait_first_plus : kind[0] == 'C' ? pred_count : NULL, &k, "Int64",
                        *mpa_pool_epoch(pool) + 1, 0, &ret);
    }
    if (rc != MPA_OK) {
      fprintf(stderr, "op %lld failed: %s\n", op, mpa_last_error());
      MPI_Abort(MPI_COMM_WORLD, 3);
    }
    if (ret != repochs) { /* the returned vector aliases the pool's (src/MPIAsyncPools.jl:187) */
      fprintf(stderr, "repochs not aliased\n");
      MPI_Abort(MPI_COMM_WORLD, 5);
    }
    for (long long i = 0; i < n; ++i) printf("%lld ", (long long)repochs[i]);
    printf("|");
    for (long long i = 0; i < n; ++i) printf(" %d", (int)active[i]);
    printf(" |");
    for (long long i = 0; i < 3 * n; ++i) printf(" %.17g", recv[i]);
    printf("\n");
  }
  fclose(f);
  /* drain, then the control tag (examples/iterative_example.jl:49-52) */
  if (mpa_waitall(pool, recv, rb, 3 * n, irecv, rb, NULL) != MPA_OK) MPI_Abort(MPI_COMM_WORLD, 3);
  for (long long r = 1; r <= n; ++r) {
    double z = 0;
    MPI_Send(&z, 1, MPI_DOUBLE, (int)r, CONTROL_TAG, MPI_COMM_WORLD);
  }
  fflush(stdout);
  mpa_comm_destroy(comm);
  mpa_pool_destroy(pool);
  free(isend);
  free(recv);
  free(irecv);
  free(dur);
  MPI_Finalize();
  return 0;
}
