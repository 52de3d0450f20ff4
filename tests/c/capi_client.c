/*
 * A C client of the C ABI (include/mpiasyncpools.h) in a process without torch: the system
 * ROCm runtime and plain hipMalloc buffers of exactly the sizes the ABI states, which is what
 * the Julia binding (julia/) gets through ccall.  (torch's caching allocator hands out slack
 * around small tensors, so an out-of-bounds read there goes unnoticed; here it faults.)
 *
 * Per case: n workers with shards of the global synthetic problem (mpa_generate), one
 * mpa_asyncmap with nwait = n, every reply chunk against g_i = A_i^T (A_i x - b_i) (or the
 * batched G_i = A_i^T (A_i X - B_i) in bf16) computed on the host in double from the device's
 * own A_i / b_i.  Then the shipped device paths beyond one call:
 *   descent  mpa_lsq_descent / mpa_lsqb_descent for several epochs (launch-ahead, the fused
 *            tail at <= 2048 columns, the separate epoch kernel for wide rows): the final
 *            iterate against a host fp64 replay of the descent (fp32 / fp64), or (bf16
 *            messages) the last replies against the host gradient of the message the device
 *            last sent and that message against the final iterate;
 *   stale    nwait < n with a gated schedule (mpa_comm_set_gate): a stale harvest in the wait
 *            loop, its held re-dispatch, a phase-1 harvest, a tie and waitall!, every reply
 *            chunk against the gradient of the iterate of its epoch, and the repochs trace.
 * Prints one line per case:
 *   case <dtype> <n> <rows> <cols> relerr <worst over workers> [descent|stale]
 * Built by tests/c/Makefile (from __graft_entry__.build()); run by tests/test_gpu_capi_client.py.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#include "mpiasyncpools.h"

#define CHECK(c)                                                       \
  do {                                                                 \
    int r_ = (c);                                                      \
    if (r_) {                                                          \
      printf("FAIL %s -> %d (%s)\n", #c, r_, mpa_last_error());        \
      exit(1);                                                         \
    }                                                                  \
  } while (0)
#define HCHECK(c)                                                      \
  do {                                                                 \
    hipError_t e_ = (c);                                               \
    if (e_) {                                                          \
      printf("FAIL %s -> %s\n", #c, hipGetErrorString(e_));            \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

static double get(const void* p, int f64, size_t k) { return f64 ? ((const double*)p)[k] : ((const float*)p)[k]; }

static double run_case(int dtype, int n, long long rows, long long cols) {
  const int f64 = dtype == MPA_F64;
  const size_t es = f64 ? 8 : 4;
  void** A = calloc((size_t)n, sizeof(void*));
  void** b = calloc((size_t)n, sizeof(void*));
  mpa_comm* comm = NULL;
  mpa_pool* pool = NULL;
  CHECK(mpa_comm_create(MPA_TRANSPORT_HIP, n, NULL, &comm));
  for (int w = 0; w < n; ++w) {
    HCHECK(hipMalloc(&A[w], es * (size_t)(rows * cols)));
    HCHECK(hipMalloc(&b[w], es * (size_t)rows));
    const unsigned long long r0 = (unsigned long long)w * (unsigned long long)rows;
    CHECK(mpa_generate(A[w], dtype, 11, 0, r0 * (unsigned long long)cols, rows * cols, 1.0 / sqrt((double)cols), NULL));
    CHECK(mpa_generate(b[w], dtype, 11, 1, r0, rows, 1.0, NULL));
    CHECK(mpa_comm_set_task_lsq(comm, w + 1, dtype, rows, cols, A[w], cols, b[w]));
  }
  HCHECK(hipDeviceSynchronize());
  CHECK(mpa_pool_create(n, NULL, 0, n, &pool));
  const size_t xb = es * (size_t)cols, rb = xb * (size_t)n;
  void *dx, *dr, *dix, *dir;
  HCHECK(hipMalloc(&dx, xb));
  HCHECK(hipMalloc(&dr, rb));
  HCHECK(hipMalloc(&dix, rb));
  HCHECK(hipMalloc(&dir, rb));
  void* x = malloc(xb);
  for (long long j = 0; j < cols; ++j) {
    const double v = 0.01 * (double)(j % 7 - 3);
    if (f64) ((double*)x)[j] = v;
    else ((float*)x)[j] = (float)v;
  }
  HCHECK(hipMemcpy(dx, x, xb, hipMemcpyHostToDevice));
  CHECK(mpa_asyncmap(pool, dx, xb, dr, rb, (size_t)(n * cols), dix, rb, dir, rb, comm, MPA_NWAIT_INT, n, NULL, NULL,
                     NULL, 1, 0, NULL));
  HCHECK(hipDeviceSynchronize());
  void* g = malloc(rb);
  HCHECK(hipMemcpy(g, dr, rb, hipMemcpyDeviceToHost));
  void* Ah = malloc(es * (size_t)(rows * cols));
  void* bh = malloc(es * (size_t)rows);
  double* ref = malloc(sizeof(double) * (size_t)cols);
  double worst = 0.0;
  for (int w = 0; w < n; ++w) {
    HCHECK(hipMemcpy(Ah, A[w], es * (size_t)(rows * cols), hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(bh, b[w], es * (size_t)rows, hipMemcpyDeviceToHost));
    memset(ref, 0, sizeof(double) * (size_t)cols);
    for (long long r = 0; r < rows; ++r) {
      double d = -get(bh, f64, (size_t)r);
      for (long long j = 0; j < cols; ++j) d += get(Ah, f64, (size_t)(r * cols + j)) * get(x, f64, (size_t)j);
      for (long long j = 0; j < cols; ++j) ref[j] += d * get(Ah, f64, (size_t)(r * cols + j));
    }
    double num = 0.0, den = 0.0;
    for (long long j = 0; j < cols; ++j) {
      const double e = get(g, f64, (size_t)(w * cols + j)) - ref[j];
      num += e * e;
      den += ref[j] * ref[j];
    }
    const double rel = sqrt(num / (den > 0 ? den : 1.0));
    if (rel > worst || rel != rel) worst = rel;
  }
  CHECK(mpa_comm_shutdown(comm));
  mpa_pool_destroy(pool);
  mpa_comm_destroy(comm);
  for (int w = 0; w < n; ++w) {
    HCHECK(hipFree(A[w]));
    HCHECK(hipFree(b[w]));
  }
  HCHECK(hipFree(dx));
  HCHECK(hipFree(dr));
  HCHECK(hipFree(dix));
  HCHECK(hipFree(dir));
  free(A);
  free(b);
  free(x);
  free(g);
  free(Ah);
  free(bh);
  free(ref);
  return worst;
}

/* the batched variant (BASELINE configs[4]): G_i = A_i^T (A_i X - B_i), bf16 A / B / X, fp32 G,
 * 64 iterates; host reference in double from the device's own bf16 bits */
static float bf(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static double run_batch(int n, long long rows, long long cols) {
  const long long K = 64;
  uint16_t** A = calloc((size_t)n, sizeof(void*));
  uint16_t** B = calloc((size_t)n, sizeof(void*));
  mpa_comm* comm = NULL;
  mpa_pool* pool = NULL;
  CHECK(mpa_comm_create(MPA_TRANSPORT_HIP, n, NULL, &comm));
  for (int w = 0; w < n; ++w) {
    HCHECK(hipMalloc((void**)&A[w], 2 * (size_t)(rows * cols)));
    HCHECK(hipMalloc((void**)&B[w], 2 * (size_t)(rows * K)));
    const unsigned long long r0 = (unsigned long long)w * (unsigned long long)rows;
    CHECK(mpa_generate(A[w], MPA_BF16, 13, 0, r0 * (unsigned long long)cols, rows * cols, 1.0 / sqrt((double)cols), NULL));
    CHECK(mpa_generate(B[w], MPA_BF16, 13, 1, r0 * (unsigned long long)K, rows * K, 1.0, NULL));
    CHECK(mpa_comm_set_task_lsq_batch(comm, w + 1, rows, cols, K, A[w], cols, B[w]));
  }
  CHECK(mpa_pool_create(n, NULL, 0, n, &pool));
  const size_t xb = 2 * (size_t)(cols * K), gb = 4 * (size_t)(cols * K);
  uint16_t *dX, *diX;
  float *dG, *diG;
  HCHECK(hipMalloc((void**)&dX, xb));
  HCHECK(hipMalloc((void**)&diX, xb * (size_t)n));
  HCHECK(hipMalloc((void**)&dG, gb * (size_t)n));
  HCHECK(hipMalloc((void**)&diG, gb * (size_t)n));
  CHECK(mpa_generate(dX, MPA_BF16, 13, 2, 0, cols * K, 0.5, NULL));
  HCHECK(hipDeviceSynchronize());
  CHECK(mpa_asyncmap(pool, dX, xb, dG, gb * (size_t)n, (size_t)(n * cols * K), diX, xb * (size_t)n, diG,
                     gb * (size_t)n, comm, MPA_NWAIT_INT, n, NULL, NULL, NULL, 1, 0, NULL));
  HCHECK(hipDeviceSynchronize());
  uint16_t* X = malloc(xb);
  float* G = malloc(gb * (size_t)n);
  uint16_t* Ah = malloc(2 * (size_t)(rows * cols));
  uint16_t* Bh = malloc(2 * (size_t)(rows * K));
  double* R = malloc(sizeof(double) * (size_t)K);
  double* ref = malloc(sizeof(double) * (size_t)(cols * K));
  HCHECK(hipMemcpy(X, dX, xb, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(G, dG, gb * (size_t)n, hipMemcpyDeviceToHost));
  double worst = 0.0;
  for (int w = 0; w < n; ++w) {
    HCHECK(hipMemcpy(Ah, A[w], 2 * (size_t)(rows * cols), hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(Bh, B[w], 2 * (size_t)(rows * K), hipMemcpyDeviceToHost));
    memset(ref, 0, sizeof(double) * (size_t)(cols * K));
    for (long long r = 0; r < rows; ++r) {
      for (long long k = 0; k < K; ++k) R[k] = -(double)bf(Bh[r * K + k]);
      for (long long j = 0; j < cols; ++j) {
        const double a = bf(Ah[r * cols + j]);
        for (long long k = 0; k < K; ++k) R[k] += a * (double)bf(X[j * K + k]);
      }
      for (long long j = 0; j < cols; ++j) {
        const double a = bf(Ah[r * cols + j]);
        for (long long k = 0; k < K; ++k) ref[j * K + k] += a * R[k];
      }
    }
    double num = 0.0, den = 0.0;
    for (long long e = 0; e < cols * K; ++e) {
      const double d = (double)G[(size_t)w * (size_t)(cols * K) + (size_t)e] - ref[e];
      num += d * d;
      den += ref[e] * ref[e];
    }
    const double rel = sqrt(num / (den > 0 ? den : 1.0));
    if (rel > worst || rel != rel) worst = rel;
  }
  CHECK(mpa_comm_shutdown(comm));
  mpa_pool_destroy(pool);
  mpa_comm_destroy(comm);
  for (int w = 0; w < n; ++w) {
    HCHECK(hipFree(A[w]));
    HCHECK(hipFree(B[w]));
  }
  HCHECK(hipFree(dX));
  HCHECK(hipFree(diX));
  HCHECK(hipFree(dG));
  HCHECK(hipFree(diG));
  free(A);
  free(B);
  free(X);
  free(G);
  free(Ah);
  free(Bh);
  free(R);
  free(ref);
  return worst;
}

/* ---- shared helpers of the multi-call cases ---------------------------------------------- */

/* host fp64 gradient of one fp32 / fp64 shard at x */
static void host_grad(int f64, const void* Ah, const void* bh, const double* x, long long rows, long long cols,
                      double* out) {
  memset(out, 0, sizeof(double) * (size_t)cols);
  for (long long r = 0; r < rows; ++r) {
    double d = -get(bh, f64, (size_t)r);
    for (long long j = 0; j < cols; ++j) d += get(Ah, f64, (size_t)(r * cols + j)) * x[j];
    for (long long j = 0; j < cols; ++j) out[j] += d * get(Ah, f64, (size_t)(r * cols + j));
  }
}

static double relerr(const double* got, const double* ref, size_t m) {
  double num = 0.0, den = 0.0;
  for (size_t j = 0; j < m; ++j) {
    num += (got[j] - ref[j]) * (got[j] - ref[j]);
    den += ref[j] * ref[j];
  }
  const double r = sqrt(num / (den > 0 ? den : 1.0));
  return r == r ? r : 1e300;
}

/* n fp32 / fp64 shards (rows x cols, exact-size hipMalloc buffers) registered on comm, with
 * host copies for the references */
typedef struct {
  int n, f64;
  long long rows, cols;
  size_t es;
  void **A, **b, **Ah, **bh;
} Shards;

static Shards shards_make(mpa_comm* comm, int dtype, int n, long long rows, long long cols, unsigned seed) {
  Shards s = {n, dtype == MPA_F64, rows, cols, dtype == MPA_F64 ? 8u : 4u, NULL, NULL, NULL, NULL};
  s.A = calloc((size_t)n, sizeof(void*));
  s.b = calloc((size_t)n, sizeof(void*));
  s.Ah = calloc((size_t)n, sizeof(void*));
  s.bh = calloc((size_t)n, sizeof(void*));
  for (int w = 0; w < n; ++w) {
    HCHECK(hipMalloc(&s.A[w], s.es * (size_t)(rows * cols)));
    HCHECK(hipMalloc(&s.b[w], s.es * (size_t)rows));
    const unsigned long long r0 = (unsigned long long)w * (unsigned long long)rows;
    CHECK(mpa_generate(s.A[w], dtype, seed, 0, r0 * (unsigned long long)cols, rows * cols, 1.0 / sqrt((double)cols), NULL));
    CHECK(mpa_generate(s.b[w], dtype, seed, 1, r0, rows, 1.0, NULL));
    CHECK(mpa_comm_set_task_lsq(comm, w + 1, dtype, rows, cols, s.A[w], cols, s.b[w]));
    s.Ah[w] = malloc(s.es * (size_t)(rows * cols));
    s.bh[w] = malloc(s.es * (size_t)rows);
    HCHECK(hipMemcpy(s.Ah[w], s.A[w], s.es * (size_t)(rows * cols), hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(s.bh[w], s.b[w], s.es * (size_t)rows, hipMemcpyDeviceToHost));
  }
  return s;
}

static void shards_free(Shards* s) {
  for (int w = 0; w < s->n; ++w) {
    HCHECK(hipFree(s->A[w]));
    HCHECK(hipFree(s->b[w]));
    free(s->Ah[w]);
    free(s->bh[w]);
  }
  free(s->A);
  free(s->b);
  free(s->Ah);
  free(s->bh);
}

/* step size 0.9 / L with L ~ ||A||^2 of the stacked shards (entries uniform on
 * [-1, 1) / sqrt(cols)), as bench.py picks it */
static double step_size(int n, long long rows, long long cols) {
  const double m = (double)n * (double)rows, c = (double)cols;
  const double s = 1.0 + sqrt(c / m);
  return 0.9 / (m / (3.0 * c) * s * s);
}

/* mpa_lsq_descent, nwait = n, `epochs` epochs from x = 0: the device iterate against a host
 * fp64 replay of the same descent, and the last replies against the host gradient at the
 * replay's last message */
static double run_descent(int dtype, int n, long long rows, long long cols, int epochs) {
  mpa_comm* comm = NULL;
  mpa_pool* pool = NULL;
  CHECK(mpa_comm_create(MPA_TRANSPORT_HIP, n, NULL, &comm));
  Shards S = shards_make(comm, dtype, n, rows, cols, 17);
  CHECK(mpa_pool_create(n, NULL, 0, n, &pool));
  const size_t xb = S.es * (size_t)cols, rb = xb * (size_t)n;
  void *dx, *dr, *dix, *dir;
  HCHECK(hipMalloc(&dx, xb));
  HCHECK(hipMalloc(&dr, rb));
  HCHECK(hipMalloc(&dix, rb));
  HCHECK(hipMalloc(&dir, rb));
  HCHECK(hipMemset(dx, 0, xb));
  HCHECK(hipDeviceSynchronize());
  const double eta = step_size(n, rows, cols);
  CHECK(mpa_lsq_descent(pool, comm, dtype, dx, cols, dr, rb, dix, rb, dir, rb, MPA_NWAIT_INT, n, NULL, NULL, eta, 0.0,
                        epochs));
  HCHECK(hipDeviceSynchronize());
  void* xd = malloc(xb);
  void* gd = malloc(rb);
  HCHECK(hipMemcpy(xd, dx, xb, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(gd, dr, rb, hipMemcpyDeviceToHost));
  double* x = calloc((size_t)cols, sizeof(double));
  double* xlast = calloc((size_t)cols, sizeof(double));
  double* g = malloc(sizeof(double) * (size_t)cols * (size_t)n);
  double* tmp = malloc(sizeof(double) * (size_t)cols);
  for (int e = 0; e < epochs; ++e) {
    memcpy(xlast, x, sizeof(double) * (size_t)cols);
    for (int w = 0; w < n; ++w) host_grad(S.f64, S.Ah[w], S.bh[w], xlast, rows, cols, g + (size_t)w * (size_t)cols);
    for (long long j = 0; j < cols; ++j) {
      double sum = 0.0;
      for (int w = 0; w < n; ++w) sum += g[(size_t)w * (size_t)cols + (size_t)j];
      x[j] = xlast[j] - eta * sum;
    }
  }
  double worst = 0.0;
  for (long long j = 0; j < cols; ++j) tmp[j] = get(xd, S.f64, (size_t)j);
  worst = relerr(tmp, x, (size_t)cols);
  for (int w = 0; w < n; ++w) {
    for (long long j = 0; j < cols; ++j) tmp[j] = get(gd, S.f64, (size_t)w * (size_t)cols + (size_t)j);
    const double e = relerr(tmp, g + (size_t)w * (size_t)cols, (size_t)cols);
    if (e > worst) worst = e;
  }
  CHECK(mpa_comm_shutdown(comm));
  mpa_pool_destroy(pool);
  mpa_comm_destroy(comm);
  shards_free(&S);
  HCHECK(hipFree(dx));
  HCHECK(hipFree(dr));
  HCHECK(hipFree(dix));
  HCHECK(hipFree(dir));
  free(xd);
  free(gd);
  free(x);
  free(xlast);
  free(g);
  free(tmp);
  return worst;
}

/* mpa_lsqb_descent (bf16 messages, fp32 iterate), nwait = n: the last replies against the
 * host gradient of the message each worker was last sent (isendbuf), and that message
 * against the final iterate: message = bf16(x_prev) with x_prev = x_final + eta sum_i G_i */
static double run_descent_batch(int n, long long rows, long long cols, int epochs) {
  const long long K = 64, elems = cols * K;
  uint16_t** A = calloc((size_t)n, sizeof(void*));
  uint16_t** B = calloc((size_t)n, sizeof(void*));
  mpa_comm* comm = NULL;
  mpa_pool* pool = NULL;
  CHECK(mpa_comm_create(MPA_TRANSPORT_HIP, n, NULL, &comm));
  for (int w = 0; w < n; ++w) {
    HCHECK(hipMalloc((void**)&A[w], 2 * (size_t)(rows * cols)));
    HCHECK(hipMalloc((void**)&B[w], 2 * (size_t)(rows * K)));
    const unsigned long long r0 = (unsigned long long)w * (unsigned long long)rows;
    CHECK(mpa_generate(A[w], MPA_BF16, 19, 0, r0 * (unsigned long long)cols, rows * cols, 1.0 / sqrt((double)cols), NULL));
    CHECK(mpa_generate(B[w], MPA_BF16, 19, 1, r0 * (unsigned long long)K, rows * K, 1.0, NULL));
    CHECK(mpa_comm_set_task_lsq_batch(comm, w + 1, rows, cols, K, A[w], cols, B[w]));
  }
  CHECK(mpa_pool_create(n, NULL, 0, n, &pool));
  const size_t xb = 2 * (size_t)elems, gb = 4 * (size_t)elems;
  float *dx32, *dG, *diG;
  uint16_t *dxb, *diX;
  HCHECK(hipMalloc((void**)&dx32, gb));
  HCHECK(hipMalloc((void**)&dxb, xb));
  HCHECK(hipMalloc((void**)&diX, xb * (size_t)n));
  HCHECK(hipMalloc((void**)&dG, gb * (size_t)n));
  HCHECK(hipMalloc((void**)&diG, gb * (size_t)n));
  HCHECK(hipMemset(dx32, 0, gb));
  HCHECK(hipMemset(dxb, 0, xb));
  HCHECK(hipDeviceSynchronize());
  const double eta = step_size(n, rows, cols);
  CHECK(mpa_lsqb_descent(pool, comm, dx32, dxb, elems, dG, gb * (size_t)n, diX, xb * (size_t)n, diG, gb * (size_t)n,
                         MPA_NWAIT_INT, n, NULL, NULL, eta, 0.0, epochs));
  HCHECK(hipDeviceSynchronize());
  uint16_t* X = malloc(xb * (size_t)n);
  float* G = malloc(gb * (size_t)n);
  float* x32 = malloc(gb);
  uint16_t* Ah = malloc(2 * (size_t)(rows * cols));
  uint16_t* Bh = malloc(2 * (size_t)(rows * K));
  double* R = malloc(sizeof(double) * (size_t)K);
  double* ref = malloc(sizeof(double) * (size_t)elems);
  double* got = malloc(sizeof(double) * (size_t)elems);
  HCHECK(hipMemcpy(X, diX, xb * (size_t)n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(G, dG, gb * (size_t)n, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(x32, dx32, gb, hipMemcpyDeviceToHost));
  double worst = 0.0;
  for (int w = 0; w < n; ++w) {
    const uint16_t* Xw = X + (size_t)w * (size_t)elems;
    if (memcmp(Xw, X, xb)) return 1.0;  /* every worker was sent the same message */
    HCHECK(hipMemcpy(Ah, A[w], 2 * (size_t)(rows * cols), hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(Bh, B[w], 2 * (size_t)(rows * K), hipMemcpyDeviceToHost));
    memset(ref, 0, sizeof(double) * (size_t)elems);
    for (long long r = 0; r < rows; ++r) {
      for (long long k = 0; k < K; ++k) R[k] = -(double)bf(Bh[r * K + k]);
      for (long long j = 0; j < cols; ++j) {
        const double a = bf(Ah[r * cols + j]);
        for (long long k = 0; k < K; ++k) R[k] += a * (double)bf(Xw[j * K + k]);
      }
      for (long long j = 0; j < cols; ++j) {
        const double a = bf(Ah[r * cols + j]);
        for (long long k = 0; k < K; ++k) ref[j * K + k] += a * R[k];
      }
    }
    for (long long e = 0; e < elems; ++e) got[e] = G[(size_t)w * (size_t)elems + (size_t)e];
    const double e = relerr(got, ref, (size_t)elems);
    if (e > worst) worst = e;
  }
  /* the message is the bf16 rounding of the iterate before the last update */
  for (long long e = 0; e < elems; ++e) {
    double sum = 0.0;
    for (int w = 0; w < n; ++w) sum += G[(size_t)w * (size_t)elems + (size_t)e];
    const double xprev = (double)x32[e] + eta * sum, m = bf(X[e]);
    if (fabs(m - xprev) > ldexp(fabs(xprev), -8) + 1e-30) {
      printf("FAIL bf16 message %lld: %.9g, iterate before the update %.9g\n", e, m, xprev);
      exit(1);
    }
  }
  CHECK(mpa_comm_shutdown(comm));
  mpa_pool_destroy(pool);
  mpa_comm_destroy(comm);
  for (int w = 0; w < n; ++w) {
    HCHECK(hipFree(A[w]));
    HCHECK(hipFree(B[w]));
  }
  HCHECK(hipFree(dx32));
  HCHECK(hipFree(dxb));
  HCHECK(hipFree(diX));
  HCHECK(hipFree(dG));
  HCHECK(hipFree(diG));
  free(A);
  free(B);
  free(X);
  free(G);
  free(x32);
  free(Ah);
  free(Bh);
  free(R);
  free(ref);
  free(got);
  return worst;
}

/* k-of-n with stale results, 3 workers, nwait 2, under a hand-written gated schedule
 * (mpa_comm_set_gate) so the order is fixed:
 *   call 1  Waitany! sees worker 1, then worker 3               -> repochs [1, 0, 1]
 *   call 2  worker 2's epoch-1 reply in the wait loop: stale, re-dispatched (held, then
 *           launched when the schedule completes it), fresh; then worker 1 -> [2, 2, 1]
 *   call 3  phase 1 harvests worker 3's epoch-2 reply; workers 1 and 2 complete together
 *           (a tie: lowest index first)                         -> [3, 3, 2]
 *   waitall! harvests worker 3                                  -> [3, 3, 3]
 * (src/MPIAsyncPools.jl:91-114,161-184,195-224).  Every reply chunk against the host
 * gradient at the iterate of its epoch, after every call. */
static double run_stale(int dtype, long long rows, long long cols) {
  const int n = 3;
  mpa_comm* comm = NULL;
  mpa_pool* pool = NULL;
  CHECK(mpa_comm_create(MPA_TRANSPORT_HIP, n, NULL, &comm));
  Shards S = shards_make(comm, dtype, n, rows, cols, 23);
  const int kinds[] = {MPA_GATE_CALL, MPA_GATE_WAIT, MPA_GATE_WAIT,                  /* call 1 */
                       MPA_GATE_CALL, MPA_GATE_WAIT, MPA_GATE_WAIT, MPA_GATE_WAIT,   /* call 2 */
                       MPA_GATE_CALL, MPA_GATE_WAIT, MPA_GATE_WAIT,                  /* call 3 */
                       MPA_GATE_WAITALL};
  const int64_t offs[] = {0, 0, 1, 2, 2, 3, 4, 5, 6, 8, 8, 9};
  const int64_t rel[] = {1, 3, 2, 2, 1, 3, 1, 2, 3};
  CHECK(mpa_comm_set_gate(comm, 11, kinds, offs, rel));
  CHECK(mpa_pool_create(n, NULL, 0, n, &pool));
  const size_t xb = S.es * (size_t)cols, rb = xb * (size_t)n;
  void *dx, *dr, *dix, *dir;
  HCHECK(hipMalloc(&dx, xb));
  HCHECK(hipMalloc(&dr, rb));
  HCHECK(hipMalloc(&dix, rb));
  HCHECK(hipMalloc(&dir, rb));
  void* xt = malloc(xb);
  void* gd = malloc(rb);
  double* xs = malloc(sizeof(double) * (size_t)cols * 4); /* the iterate of epochs 1..3 */
  double* ref = malloc(sizeof(double) * (size_t)cols);
  double* got = malloc(sizeof(double) * (size_t)cols);
  const int64_t want[4][3] = {{1, 0, 1}, {2, 2, 1}, {3, 3, 2}, {3, 3, 3}};
  double worst = 0.0;
  for (int call = 0; call < 4; ++call) {
    int64_t* rep = NULL;
    if (call < 3) {
      const int epoch = call + 1;
      for (long long j = 0; j < cols; ++j) {
        const double v = 0.01 * (double)epoch * (double)(j % 7 - 3) + 0.001 * (double)epoch;
        xs[(size_t)epoch * (size_t)cols + (size_t)j] = S.f64 ? v : (double)(float)v;
        if (S.f64) ((double*)xt)[j] = v;
        else ((float*)xt)[j] = (float)v;
      }
      HCHECK(hipMemcpy(dx, xt, xb, hipMemcpyHostToDevice));
      CHECK(mpa_asyncmap(pool, dx, xb, dr, rb, (size_t)(n * cols), dix, rb, dir, rb, comm, MPA_NWAIT_INT, 2, NULL, NULL,
                         NULL, epoch, 0, &rep));
    } else {
      CHECK(mpa_waitall(pool, dr, rb, (size_t)(n * cols), dir, rb, &rep));
    }
    HCHECK(hipDeviceSynchronize());
    for (int i = 0; i < n; ++i)
      if (rep[i] != want[call][i]) {
        printf("FAIL stale case, call %d: repochs[%d] = %lld, want %lld\n", call + 1, i, (long long)rep[i],
               (long long)want[call][i]);
        exit(1);
      }
    HCHECK(hipMemcpy(gd, dr, rb, hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) {
      if (rep[i] == 0) continue;
      host_grad(S.f64, S.Ah[i], S.bh[i], xs + (size_t)rep[i] * (size_t)cols, rows, cols, ref);
      for (long long j = 0; j < cols; ++j) got[j] = get(gd, S.f64, (size_t)i * (size_t)cols + (size_t)j);
      const double e = relerr(got, ref, (size_t)cols);
      if (e > worst) worst = e;
    }
  }
  if (mpa_comm_counter(comm, "held") != 1 || mpa_comm_counter(comm, "gate_steps") != 11) {
    printf("FAIL stale case: held %lld (want 1), gate steps %lld (want 11)\n", (long long)mpa_comm_counter(comm, "held"),
           (long long)mpa_comm_counter(comm, "gate_steps"));
    exit(1);
  }
  CHECK(mpa_comm_shutdown(comm));
  mpa_pool_destroy(pool);
  mpa_comm_destroy(comm);
  shards_free(&S);
  HCHECK(hipFree(dx));
  HCHECK(hipFree(dr));
  HCHECK(hipFree(dix));
  HCHECK(hipFree(dir));
  free(xt);
  free(gd);
  free(xs);
  free(ref);
  free(got);
  return worst;
}

int main(void) {
  HCHECK(hipSetDevice(0));
  /* narrow rows whose last 16-B vectors lie past cols (one vector per lane and fewer than 64
   * valid), a full-width narrow row, and wide rows with a short last slice */
  const struct { int dtype, n; long long rows, cols; } cases[] = {
      {MPA_F64, 1, 4096, 64}, {MPA_F64, 3, 4096, 64}, {MPA_F32, 1, 1000, 100}, {MPA_F32, 2, 17, 8},
      {MPA_F32, 1, 3000, 1024}, {MPA_F64, 1, 333, 2050}, {MPA_F32, 1, 257, 4100},
  };
  for (size_t k = 0; k < sizeof cases / sizeof cases[0]; ++k) {
    const double e = run_case(cases[k].dtype, cases[k].n, cases[k].rows, cases[k].cols);
    printf("case %s %d %lld %lld relerr %.3e\n", cases[k].dtype == MPA_F64 ? "f64" : "f32", cases[k].n,
           cases[k].rows, cases[k].cols, e);
    fflush(stdout);
  }
  /* batched bf16 (lsqp4): ragged last block, a wave with one 32-column strip (544), the
   * narrowest width, full width */
  const struct { int n; long long rows, cols; } bcases[] = {{1, 1000, 544}, {2, 77, 32}, {1, 300, 2048}};
  for (size_t k = 0; k < sizeof bcases / sizeof bcases[0]; ++k) {
    const double e = run_batch(bcases[k].n, bcases[k].rows, bcases[k].cols);
    printf("case bf16 %d %lld %lld relerr %.3e\n", bcases[k].n, bcases[k].rows, bcases[k].cols, e);
    fflush(stdout);
  }
  /* two-pass batched kernels (2048 < cols <= 4096) */
  const struct { int n; long long rows, cols; } wcases[] = {{1, 300, 4096}, {2, 129, 2080}};
  for (size_t k = 0; k < sizeof wcases / sizeof wcases[0]; ++k) {
    const double e = run_batch(wcases[k].n, wcases[k].rows, wcases[k].cols);
    printf("case bf16 %d %lld %lld relerr %.3e\n", wcases[k].n, wcases[k].rows, wcases[k].cols, e);
    fflush(stdout);
  }
  /* native descent loops: fused tail (narrow fp32 / fp64), epoch kernel (wide), bf16 messages */
  const struct { int dtype, n; long long rows, cols; int epochs; } dcases[] = {
      {MPA_F32, 4, 3000, 1024, 5}, {MPA_F64, 3, 1000, 256, 5}, {MPA_F32, 2, 500, 4096, 4}, {MPA_F64, 2, 300, 130, 6}};
  for (size_t k = 0; k < sizeof dcases / sizeof dcases[0]; ++k) {
    const double e = run_descent(dcases[k].dtype, dcases[k].n, dcases[k].rows, dcases[k].cols, dcases[k].epochs);
    printf("case %s %d %lld %lld relerr %.3e descent\n", dcases[k].dtype == MPA_F64 ? "f64" : "f32", dcases[k].n,
           dcases[k].rows, dcases[k].cols, e);
    fflush(stdout);
  }
  {
    const double e = run_descent_batch(3, 700, 512, 4);
    printf("case bf16 3 700 512 relerr %.3e descent\n", e);
    fflush(stdout);
  }
  /* k-of-n with a stale harvest, a held re-dispatch, a phase-1 harvest, a tie, waitall! */
  const struct { int dtype; long long rows, cols; } scases[] = {{MPA_F32, 2000, 300}, {MPA_F64, 1500, 130}};
  for (size_t k = 0; k < sizeof scases / sizeof scases[0]; ++k) {
    const double e = run_stale(scases[k].dtype, scases[k].rows, scases[k].cols);
    printf("case %s 3 %lld %lld relerr %.3e stale\n", scases[k].dtype == MPA_F64 ? "f64" : "f32", scases[k].rows,
           scases[k].cols, e);
    fflush(stdout);
  }
  printf("ok\n");
  return 0;
}
