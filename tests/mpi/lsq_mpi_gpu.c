/*
 * TEST DRIVER: examples/iterative_example.jl's program shape (rank 0 coordinator, ranks 1..n
 * workers, a data tag and a control tag, :1-99) with the PRODUCT pool over a real MPI
 * communicator (libmpiasyncpools_mpi.so) and worker ranks that compute their shard of the
 * least-squares gradient g_i = A_i^T (A_i x - b_i) on the GPU through the device library
 * (libmpiasyncpools.so: a one-worker HIP communicator per rank, lsq_grad_kernel in fp64):
 * BASELINE configs[0] (3 workers, fp64, A 3*2^12 x 64, nwait 2) with the compute the
 * example only simulates (`sleep(rand())`, :71) put on the device.
 *
 * Coordinator (:17-53): per epoch x -> sendbuf, repochs = asyncmap!(...; epoch, nwait),
 * then the fresh replies (repochs[i] == epoch) update x -= eta * sum_i g_i (fixed order);
 * prints "E <epoch> | <repochs>" per epoch and "X <x>" at the end, then waitall! and the
 * control-tag shutdown (:49-52).  Worker (:55-82): Irecv! on the control and data tags,
 * Waitany!, an injected host delay from argv's schedule (the straggler), the device
 * gradient, Send to the coordinator with the message's tag.
 *
 * argv: epochs nwait rows_per_worker cols seed eta delay_ms_w1,delay_ms_w2,... (per worker
 * a list cycled over its tasks, ':' between workers, e.g. "1,9:5:9,1")
 */
#define _GNU_SOURCE
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mpiasyncpools_mpi.h"

enum { DATA_TAG = 0, CONTROL_TAG = 999 };

#define CHECK(call)                                                                          \
  do {                                                                                       \
    int rc_ = (call);                                                                        \
    if (rc_) {                                                                               \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #call, rc_, mpa_last_error()); \
      MPI_Abort(MPI_COMM_WORLD, 3);                                                          \
    }                                                                                        \
  } while (0)
#define HCHECK(call)                                                      \
  do {                                                                    \
    hipError_t e_ = (call);                                               \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
      MPI_Abort(MPI_COMM_WORLD, 4);                                       \
    }                                                                     \
  } while (0)

/* this worker's delays (ms), cycled over its tasks: field `rank` of "a,b:c:d,e" */
static int parse_delays(const char* spec, int rank, double* out, int cap) {
  const char* p = spec;
  for (int r = 1; r < rank && p; ++r) {
    p = strchr(p, ':');
    if (p) ++p;
  }
  int n = 0;
  while (p && *p && *p != ':' && n < cap) {
    out[n++] = strtod(p, (char**)&p);
    if (*p == ',') ++p;
  }
  if (n == 0) out[n++] = 0.0;
  return n;
}

static void worker(int rank, int64_t rows, int64_t cols, uint64_t seed, const char* dspec) {
  double delays[64];
  const int nd = parse_delays(dspec, rank, delays, 64);
  HCHECK(hipSetDevice(0));
  double *A, *b, *dx, *dg, *dix, *dig;
  HCHECK(hipMalloc((void**)&A, sizeof(double) * (size_t)(rows * cols)));
  HCHECK(hipMalloc((void**)&b, sizeof(double) * (size_t)rows));
  const size_t xb = sizeof(double) * (size_t)cols;
  HCHECK(hipMalloc((void**)&dx, xb));
  HCHECK(hipMalloc((void**)&dg, xb));
  HCHECK(hipMalloc((void**)&dix, xb));
  HCHECK(hipMalloc((void**)&dig, xb));
  /* rows [(rank-1) rows, rank rows) of the global synthetic problem */
  const uint64_t r0 = (uint64_t)(rank - 1) * (uint64_t)rows;
  CHECK(mpa_generate(A, MPA_F64, seed, 0, r0 * (uint64_t)cols, rows * cols, 1.0 / sqrt((double)cols), NULL));
  CHECK(mpa_generate(b, MPA_F64, seed, 1, r0, rows, 1.0, NULL));
  HCHECK(hipDeviceSynchronize());
  mpa_comm* dc = NULL;
  mpa_pool* pool = NULL;
  CHECK(mpa_comm_create(MPA_TRANSPORT_HIP, 1, NULL, &dc));
  CHECK(mpa_comm_set_task_lsq(dc, 1, MPA_F64, rows, cols, A, cols, b));
  CHECK(mpa_pool_create(1, NULL, 0, 1, &pool));
  double* x = (double*)malloc(xb);
  double* g = (double*)malloc(xb);
  double ctrl = 0;
  MPI_Request rq[2];
  MPI_Irecv(&ctrl, 1, MPI_DOUBLE, 0, CONTROL_TAG, MPI_COMM_WORLD, &rq[0]); /* :61 */
  for (int64_t t = 0;; ++t) {
    MPI_Irecv(x, (int)cols, MPI_DOUBLE, 0, DATA_TAG, MPI_COMM_WORLD, &rq[1]);
    int idx = -1;
    MPI_Status st;
    MPI_Waitany(2, rq, &idx, &st); /* :72 */
    if (idx == 0) {
      MPI_Cancel(&rq[1]);
      MPI_Wait(&rq[1], MPI_STATUS_IGNORE);
      break;
    }
    const double d = delays[t % nd];
    const struct timespec ts = {(time_t)(d / 1000), (long)(fmod(d, 1000.0) * 1e6)};
    nanosleep(&ts, NULL);
    HCHECK(hipMemcpy(dx, x, xb, hipMemcpyHostToDevice));
    CHECK(mpa_asyncmap(pool, dx, xb, dg, xb, (size_t)cols, dix, xb, dig, xb, dc, MPA_NWAIT_INT, 1, NULL, NULL, NULL,
                       t + 1, 0, NULL));
    HCHECK(hipDeviceSynchronize());
    HCHECK(hipMemcpy(g, dg, xb, hipMemcpyDeviceToHost));
    MPI_Send(g, (int)cols, MPI_DOUBLE, 0, st.MPI_TAG, MPI_COMM_WORLD);
  }
  CHECK(mpa_comm_shutdown(dc));
  mpa_pool_destroy(pool);
  mpa_comm_destroy(dc);
  free(x);
  free(g);
  HCHECK(hipFree(A));
  HCHECK(hipFree(b));
  HCHECK(hipFree(dx));
  HCHECK(hipFree(dg));
  HCHECK(hipFree(dix));
  HCHECK(hipFree(dig));
}

static void coordinator(int64_t n, int64_t epochs, int64_t nwait, int64_t cols, double eta) {
  mpa_comm* mc = NULL;
  mpa_pool* pool = NULL;
  CHECK(mpa_comm_create_mpi((int64_t)MPI_Comm_c2f(MPI_COMM_WORLD), &mc));
  CHECK(mpa_pool_create(n, NULL, 0, nwait, &pool));
  const size_t xb = sizeof(double) * (size_t)cols, rb = xb * (size_t)n;
  double* x = (double*)calloc((size_t)cols, sizeof(double));
  double* send = (double*)malloc(xb);
  double* isend = (double*)malloc(rb);
  double* recv = (double*)calloc((size_t)(n * cols), sizeof(double));
  double* irecv = (double*)calloc((size_t)(n * cols), sizeof(double));
  for (int64_t epoch = 1; epoch <= epochs; ++epoch) {
    memcpy(send, x, xb);
    int64_t* rep = NULL;
    CHECK(mpa_asyncmap(pool, send, xb, recv, rb, (size_t)(n * cols), isend, rb, irecv, rb, mc, MPA_NWAIT_INT, nwait,
                       NULL, NULL, NULL, epoch, DATA_TAG, &rep));
    printf("E %lld |", (long long)epoch);
    for (int64_t i = 0; i < n; ++i) printf(" %lld", (long long)rep[i]);
    printf("\n");
    for (int64_t j = 0; j < cols; ++j) { /* x -= eta * sum of the fresh replies, workers in order */
      double s = 0.0;
      for (int64_t i = 0; i < n; ++i)
        if (rep[i] == epoch) s += recv[i * cols + j];
      x[j] -= eta * s;
    }
  }
  printf("X");
  for (int64_t j = 0; j < cols; ++j) printf(" %.17g", x[j]);
  printf("\n");
  fflush(stdout);
  CHECK(mpa_waitall(pool, recv, rb, (size_t)(n * cols), irecv, rb, NULL));
  double z = 0.0;
  for (int64_t i = 1; i <= n; ++i) MPI_Send(&z, 1, MPI_DOUBLE, (int)i, CONTROL_TAG, MPI_COMM_WORLD); /* :49-52 */
  mpa_pool_destroy(pool);
  mpa_comm_destroy(mc);
  free(x);
  free(send);
  free(isend);
  free(recv);
  free(irecv);
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank = 0, size = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  if (argc < 8 || size < 2) {
    if (rank == 0) fprintf(stderr, "usage: mpiexec -n <n+1> lsq_mpi_gpu epochs nwait rows cols seed eta delays\n");
    MPI_Abort(MPI_COMM_WORLD, 2);
  }
  const int64_t epochs = atoll(argv[1]), nwait = atoll(argv[2]), rows = atoll(argv[3]), cols = atoll(argv[4]);
  const uint64_t seed = strtoull(argv[5], NULL, 10);
  const double eta = strtod(argv[6], NULL);
  if (rank == 0) coordinator(size - 1, epochs, nwait, cols, eta);
  else worker(rank, rows, cols, seed, argv[7]);
  MPI_Barrier(MPI_COMM_WORLD); /* :99 */
  MPI_Finalize();
  return 0;
}
