/*
 * A C client of the C ABI (include/mpiasyncpools.h) in a process without torch: the system
 * ROCm runtime and plain hipMalloc buffers of exactly the sizes the ABI states, which is what
 * the Julia binding (julia/) gets through ccall.  (torch's caching allocator hands out slack
 * around small tensors, so an out-of-bounds read there goes unnoticed; here it faults.)
 *
 * Per case: n workers with shards of the global synthetic problem (mpa_generate), one
 * mpa_asyncmap with nwait = n, every reply chunk against g_i = A_i^T (A_i x - b_i) (or the
 * batched G_i = A_i^T (A_i X - B_i) in bf16) computed on the host in double from the device's
 * own A_i / b_i.  Prints one line per case:
 *   case <dtype> <n> <rows> <cols> relerr <worst over workers>
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
  printf("ok\n");
  return 0;
}
