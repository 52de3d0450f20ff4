/*
 * ORACLE / CPU BASELINE — TEST AND MEASUREMENT INFRASTRUCTURE ONLY.
 *
 * The reference's coordinator + worker programs on host cores: the C restatement of
 * src/MPIAsyncPools.jl (asyncpool_oracle.c, the same state machine) driving n worker
 * threads through a shared-memory transport that has MPI's Isend/Irecv!/Test!/Waitany!/
 * Waitall! semantics (one outstanding message per worker, FIFO replies,
 * examples/iterative_example.jl:55-82).  Each worker computes the BASELINE workload
 * g_i = A_i^T (A_i x - b_i) in fp32 on its row shard (single-threaded, AVX2 via -O3),
 * and the coordinator runs the least-squares loop of the bench
 * (asyncmap!(nwait=k); x -= eta * sum of fresh g_i).
 *
 * The real reference (Julia + MPI.jl) is not installed on this image, so bench.py reports
 * this program as cpu_baseline.kind = "port".  Data: the Philox layout of philox.h.
 *
 * usage: cpu_baseline --workers N --rows R --cols D --nwait K --seconds S [--seed X]
 *                     [--max-epochs E]
 * prints one JSON line.
 */
#include <immintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "asyncpool_oracle.h"
#include "philox.h"

static uint64_t now_ns(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

typedef struct {
  int id;
  int64_t rows, cols, row0;
  uint64_t seed;
  float* A;
  float* b;
  float* x;       /* the worker's receive buffer (MPI.Irecv! target on the worker) */
  float* g;
  _Atomic uint64_t posted;  /* tasks posted by the coordinator */
  _Atomic uint64_t done;    /* tasks replied */
  _Atomic int quit;
  uint8_t* reply_to;        /* irecvbufs[i] of the outstanding request */
  size_t sl, rl;
  pthread_t th;
} worker_t;

static void shard_gradient(const worker_t* w) {
  const int64_t d = w->cols;
  float* g = w->g;
  memset(g, 0, (size_t)d * sizeof(float));
  for (int64_t r = 0; r < w->rows; ++r) {
    const float* a = w->A + r * d;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int64_t c = 0;
    for (; c + 8 <= d; c += 8)
      for (int k = 0; k < 8; ++k) acc[k] += a[c + k] * w->x[c + k];
    float dot = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    for (; c < d; ++c) dot += a[c] * w->x[c];
    const float res = dot - w->b[r];
    for (c = 0; c < d; ++c) g[c] += res * a[c];
  }
}

static void* worker_main(void* arg) {
  worker_t* w = (worker_t*)arg;
  /* generate the shard (first touch on this thread) */
  const float scale = (float)(1.0 / sqrt((double)w->cols));
  for (int64_t r = 0; r < w->rows; ++r) {
    for (int64_t c = 0; c < w->cols; ++c)
      w->A[r * w->cols + c] = orc_unit_f32(orc_philox_word(w->seed, 0, (uint64_t)(w->row0 + r) * (uint64_t)w->cols + (uint64_t)c)) * scale;
    w->b[r] = orc_unit_f32(orc_philox_word(w->seed, 1, (uint64_t)(w->row0 + r)));
  }
  atomic_store(&w->done, 0);
  uint64_t served = 0;
  for (;;) {
    uint64_t p;
    while ((p = atomic_load_explicit(&w->posted, memory_order_acquire)) == served) {
      if (atomic_load(&w->quit)) return NULL;
      _mm_pause();
    }
    served = p;
    shard_gradient(w);
    memcpy(w->reply_to, w->g, w->rl < (size_t)w->cols * 4 ? w->rl : (size_t)w->cols * 4);
    atomic_store_explicit(&w->done, served, memory_order_release);  /* MPI.Isend reply */
  }
}

typedef struct {
  int n;
  worker_t* w;
} shm_transport;

static void t_post(void* ctx, int64_t i, int64_t rank, const uint8_t* sbuf, size_t sl, uint8_t* rbuf, size_t rl,
                   int64_t tag) {
  (void)rank; (void)tag;
  shm_transport* t = (shm_transport*)ctx;
  worker_t* w = &t->w[i];
  memcpy(w->x, sbuf, sl < (size_t)w->cols * 4 ? sl : (size_t)w->cols * 4);
  w->reply_to = rbuf;
  w->sl = sl;
  w->rl = rl;
  atomic_fetch_add_explicit(&w->posted, 1, memory_order_release);
}
static int t_test(void* ctx, int64_t i) {
  shm_transport* t = (shm_transport*)ctx;
  return atomic_load_explicit(&t->w[i].done, memory_order_acquire) == atomic_load(&t->w[i].posted);
}
static int64_t t_waitany(void* ctx, int64_t n, const uint8_t* live) {
  int any = 0;
  for (int64_t i = 0; i < n; ++i) any |= live[i];
  if (!any) return -1;
  for (;;) {
    for (int64_t i = 0; i < n; ++i)
      if (live[i] && t_test(ctx, i)) return i;
    _mm_pause();
  }
}
static void t_waitall(void* ctx, int64_t n, const uint8_t* live) {
  for (int64_t i = 0; i < n; ++i)
    while (live[i] && !t_test(ctx, i)) _mm_pause();
}
static uint64_t t_time(void* ctx) { (void)ctx; return now_ns(); }

int main(int argc, char** argv) {
  int n = 8, nwait = 8;
  int64_t rows = 1 << 20, cols = 1024, max_epochs = 1000000;
  double seconds = 10.0;
  uint64_t seed = 1234;
  for (int a = 1; a + 1 < argc; a += 2) {
    if (!strcmp(argv[a], "--workers")) n = atoi(argv[a + 1]);
    else if (!strcmp(argv[a], "--rows")) rows = atoll(argv[a + 1]);
    else if (!strcmp(argv[a], "--cols")) cols = atoll(argv[a + 1]);
    else if (!strcmp(argv[a], "--nwait")) nwait = atoi(argv[a + 1]);
    else if (!strcmp(argv[a], "--seconds")) seconds = atof(argv[a + 1]);
    else if (!strcmp(argv[a], "--seed")) seed = strtoull(argv[a + 1], NULL, 10);
    else if (!strcmp(argv[a], "--max-epochs")) max_epochs = atoll(argv[a + 1]);
  }
  const int64_t per = rows / n;
  worker_t* w = (worker_t*)calloc((size_t)n, sizeof(worker_t));
  for (int i = 0; i < n; ++i) {
    w[i].id = i;
    w[i].rows = per;
    w[i].cols = cols;
    w[i].row0 = (int64_t)i * per;
    w[i].seed = seed;
    w[i].A = (float*)aligned_alloc(64, (size_t)per * (size_t)cols * sizeof(float));
    w[i].b = (float*)aligned_alloc(64, (size_t)per * sizeof(float) + 64);
    w[i].x = (float*)aligned_alloc(64, (size_t)cols * sizeof(float) + 64);
    w[i].g = (float*)aligned_alloc(64, (size_t)cols * sizeof(float) + 64);
    atomic_store(&w[i].done, 1);  /* "generating" sentinel */
    pthread_create(&w[i].th, NULL, worker_main, &w[i]);
  }
  for (int i = 0; i < n; ++i)
    while (atomic_load(&w[i].done) != 0) _mm_pause();

  shm_transport st = {n, w};
  orc_transport tp = {&st, t_post, t_test, t_waitany, t_waitall, t_time, NULL};
  orc_pool* pool = orc_pool_create(n, NULL, 0, nwait);
  float* x = (float*)calloc((size_t)cols, sizeof(float));
  float* isend = (float*)calloc((size_t)n * (size_t)cols, sizeof(float));
  float* recv = (float*)calloc((size_t)n * (size_t)cols, sizeof(float));
  float* irecv = (float*)calloc((size_t)n * (size_t)cols, sizeof(float));
  double* acc = (double*)calloc((size_t)cols, sizeof(double));
  /* step 0.9/L with L ~ ||A||^2 for U(-1,1)/sqrt(cols) entries */
  const double L = (double)rows / (3.0 * (double)cols) * pow(1.0 + sqrt((double)cols / (double)rows), 2.0);
  const double eta = 0.9 / L;
  const size_t sl = (size_t)cols * 4, tot = (size_t)n * (size_t)cols * 4;

  int64_t epochs = 0;
  const uint64_t t0 = now_ns();
  while (epochs < max_epochs) {
    int rc = orc_asyncmap(pool, &tp, (const uint8_t*)x, sl, (uint8_t*)recv, tot, (size_t)n * (size_t)cols,
                          (uint8_t*)isend, tot, (uint8_t*)irecv, tot, ORC_NWAIT_INT, nwait, NULL, NULL, NULL,
                          pool->epoch + 1, 0);
    if (rc) { fprintf(stderr, "asyncmap failed: %s\n", pool->errmsg); return 1; }
    memset(acc, 0, (size_t)cols * sizeof(double));
    int fresh = 0;
    for (int i = 0; i < n; ++i)
      if (pool->repochs[i] == pool->epoch) {
        ++fresh;
        for (int64_t c = 0; c < cols; ++c) acc[c] += recv[(size_t)i * (size_t)cols + (size_t)c];
      }
    const double s = fresh ? eta * (double)n / (double)fresh : 0.0;
    for (int64_t c = 0; c < cols; ++c) x[c] = (float)((double)x[c] - s * acc[c]);
    ++epochs;
    if ((double)(now_ns() - t0) * 1e-9 >= seconds) break;
  }
  const double el = (double)(now_ns() - t0) * 1e-9;
  orc_waitall(pool, &tp, (uint8_t*)recv, tot, (size_t)n * (size_t)cols, (uint8_t*)irecv, tot);
  for (int i = 0; i < n; ++i) { atomic_store(&w[i].quit, 1); pthread_join(w[i].th, NULL); }
  const double bytes = (double)rows * (double)cols * 4.0 + (double)rows * 4.0 + (double)n * 2.0 * (double)sl;
  printf("{\"epochs\": %lld, \"seconds\": %.6f, \"it_per_s\": %.6f, \"alg_GBps\": %.3f, \"threads\": %d, "
         "\"workers\": %d, \"rows\": %lld, \"cols\": %lld, \"nwait\": %d, \"x0\": %.9g}\n",
         (long long)epochs, el, (double)epochs / el, bytes * (double)epochs / el / 1e9, n + 1, n,
         (long long)rows, (long long)cols, nwait, (double)x[0]);
  orc_pool_destroy(pool);
  return 0;
}
