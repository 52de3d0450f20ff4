// Store width into fine-grained device memory (the remote worker's message slot of the
// multi-process path is a fine-grained allocation exported by HIP IPC):
// the epoch step's bf16 message as 2-byte element stores (round 4: lane l stores elements
// 4l .. 4l + 3 one by one), as 8-byte and as 16-byte vector stores, into fine-grained and into
// ordinary (coarse-grained) memory.  Seven destinations of 256 KiB (c5: 2048 x 64 bf16 per
// worker) per launch, one launch = one epoch's broadcast.  Prints us per launch and GB/s.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/probe_fg_store tools/probe_fg_store.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

constexpr int kDst = 7;
constexpr int kElems = 2048 * 64;  // bf16 elements per message

struct Dsts {
  uint16_t* d[kDst];
};

// W elements per thread; MODE 0: element stores, 1: one vector store of W * 2 bytes
template <int W, int MODE>
__global__ void __launch_bounds__(256) store_kernel(const float* __restrict__ x, Dsts dst) {
  const int j = (blockIdx.x * 256 + threadIdx.x) * W;
  if (j >= kElems) return;
  uint16_t h[W];
#pragma unroll
  for (int e = 0; e < W; ++e) {
    const unsigned u = __float_as_uint(x[j + e]);
    h[e] = uint16_t((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
  }
  for (int d = 0; d < kDst; ++d) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int e = 0; e < W; ++e) dst.d[d][j + e] = h[e];
    } else if constexpr (W == 4) {
      *reinterpret_cast<uint2*>(dst.d[d] + j) = make_uint2(h[0] | (unsigned(h[1]) << 16), h[2] | (unsigned(h[3]) << 16));
    } else {
      *reinterpret_cast<uint4*>(dst.d[d] + j) = make_uint4(h[0] | (unsigned(h[1]) << 16), h[2] | (unsigned(h[3]) << 16),
                                                           h[4] | (unsigned(h[5]) << 16), h[6] | (unsigned(h[7]) << 16));
    }
  }
}

// the step's reply gather: kDst chunks of kElems fp32 read with 16-B loads, summed per element
__global__ void __launch_bounds__(256) gather_kernel(Dsts src, float* __restrict__ out) {
  const int j = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (j >= kElems) return;  // each chunk holds kElems fp32 = 512 KiB
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int d = 0; d < kDst; ++d) {
    const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(src.d[d]) + j);
    s.x += v.x, s.y += v.y, s.z += v.z, s.w += v.w;
  }
  *reinterpret_cast<float4*>(out + j) = s;
}

static double run_gather(const Dsts& d, float* out, hipStream_t s, int reps) {
  const int grid = (kElems / 4 + 255) / 256;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(gather_kernel, dim3(grid), dim3(256), 0, s, d, out);
  CK(hipEventRecord(a, s));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(gather_kernel, dim3(grid), dim3(256), 0, s, d, out);
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return double(ms) * 1e3 / reps;
}

template <int W, int MODE>
static double run(const float* x, const Dsts& d, hipStream_t s, int reps) {
  const int grid = (kElems / W + 255) / 256;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL((store_kernel<W, MODE>), dim3(grid), dim3(256), 0, s, x, d);
  CK(hipEventRecord(a, s));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((store_kernel<W, MODE>), dim3(grid), dim3(256), 0, s, x, d);
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return double(ms) * 1e3 / reps;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* x;
  CK(hipMalloc(&x, kElems * sizeof(float)));
  CK(hipMemset(x, 0x3c, kElems * sizeof(float)));
  const double bytes = double(kDst) * kElems * 2;
  for (int fine = 0; fine < 2; ++fine) {
    Dsts d;
    for (int k = 0; k < kDst; ++k) {
      if (fine) CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&d.d[k]), kElems * 2, hipDeviceMallocFinegrained));
      else CK(hipMalloc(&d.d[k], kElems * 2));
    }
    const char* kind = fine ? "fine-grained" : "coarse-grained";
    const double t0 = run<4, 0>(x, d, s, 200), t1 = run<4, 1>(x, d, s, 200), t2 = run<8, 1>(x, d, s, 200);
    std::printf("%-15s 2-B element stores %7.2f us (%6.1f GB/s) | 8-B vectors %7.2f us (%6.1f GB/s) | 16-B vectors %7.2f us (%6.1f GB/s)\n",
                kind, t0, bytes / t0 / 1e3, t1, bytes / t1 / 1e3, t2, bytes / t2 / 1e3);
    for (int k = 0; k < kDst; ++k) CK(hipFree(d.d[k]));
    // the reply gather: 7 chunks of 512 KiB fp32 (c5's reply per worker) read from this kind of memory
    Dsts g;
    for (int k = 0; k < kDst; ++k) {
      if (fine) CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&g.d[k]), kElems * 4, hipDeviceMallocFinegrained));
      else CK(hipMalloc(&g.d[k], kElems * 4));
      CK(hipMemset(g.d[k], 0, kElems * 4));
    }
    float* out;
    CK(hipMalloc(&out, kElems * 4));
    const double tg = run_gather(g, out, s, 200);
    std::printf("%-15s reply gather (7 x 512 KiB fp32, 16-B loads) %7.2f us (%6.1f GB/s read)\n", kind, tg,
                double(kDst) * kElems * 4 / tg / 1e3);
    for (int k = 0; k < kDst; ++k) CK(hipFree(g.d[k]));
    CK(hipFree(out));
  }
  CK(hipFree(x));
  return 0;
}
