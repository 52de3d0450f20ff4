// Probe of the HIP primitives the asyncmap! transport is built on (gfx950).
// Measures: kernel->host completion-flag latency, hipEventQuery cost, HBM streaming
// rate of a float4 read, aggregate rate of 8 concurrent per-worker streams,
// s_memrealtime tick rate. Not product code; results feed DESIGN.md.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include <atomic>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)
using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

__global__ void flag_kernel(volatile unsigned long long* flag, unsigned long long v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store((unsigned long long*)flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
__global__ void stream_sum(const float4* __restrict__ a, size_t n4, float* out) {
  float acc = 0.f;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = a[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678f) out[0] = acc;
}
__global__ void realtime_kernel(unsigned long long* out, int spin_us) {
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long c0 = __builtin_amdgcn_s_memtime();
  unsigned long long t1 = t0;
  while (true) { t1 = __builtin_amdgcn_s_memrealtime(); if (t1 - t0 >= (unsigned long long)spin_us * 100) break; __builtin_amdgcn_s_sleep(2); }
  unsigned long long c1 = __builtin_amdgcn_s_memtime();
  out[0] = t1 - t0; out[1] = c1 - c0;
}
int main() {
  int dev = 0; CK(hipSetDevice(dev));
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, dev));
  printf("device %s arch %s CUs %d\n", p.name, p.gcnArchName, p.multiProcessorCount);
  int wv = 0; hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, dev);
  printf("canUseStreamWaitValue %d\n", wv);
  // 1. flag latency
  unsigned long long* hflag; CK(hipHostMalloc((void**)&hflag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  *hflag = 0;
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, hflag, 0ull); CK(hipStreamSynchronize(s));
  std::vector<double> lat;
  for (int it = 1; it <= 200; ++it) {
    auto t0 = clk::now();
    hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, hflag, (unsigned long long)it);
    auto t1 = clk::now();
    while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != (unsigned long long)it) {}
    auto t2 = clk::now();
    lat.push_back(us(t0, t2));
    if (it == 200) printf("launch call %.2f us, launch->flag seen %.2f us\n", us(t0, t1), us(t0, t2));
  }
  std::sort(lat.begin(), lat.end()); printf("flag latency median %.2f us p10 %.2f p90 %.2f\n", lat[100], lat[20], lat[180]);
  CK(hipStreamSynchronize(s));
  // event query cost
  hipEvent_t ev; CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventRecord(ev, s)); CK(hipStreamSynchronize(s));
  auto q0 = clk::now(); for (int i = 0; i < 10000; ++i) (void)hipEventQuery(ev); auto q1 = clk::now();
  printf("hipEventQuery cost %.3f us\n", us(q0, q1) / 10000);
  // launch + event record + event query until done
  lat.clear();
  for (int it = 0; it < 200; ++it) {
    auto t0 = clk::now();
    hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, hflag, 0ull);
    CK(hipEventRecord(ev, s));
    while (hipEventQuery(ev) != hipSuccess) {}
    lat.push_back(us(t0, clk::now()));
  }
  std::sort(lat.begin(), lat.end()); printf("launch+event poll median %.2f us\n", lat[100]);
  // 2. HBM streaming 4 GiB
  size_t bytes = 4ull << 30; float4* a; CK(hipMalloc(&a, bytes)); CK(hipMemset(a, 0, bytes));
  float* out; CK(hipMalloc(&out, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int grid : {1024, 2048, 4096, 8192}) {
    hipLaunchKernelGGL(stream_sum, dim3(grid), dim3(256), 0, s, a, bytes / 16, out);
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(stream_sum, dim3(grid), dim3(256), 0, s, a, bytes / 16, out);
    CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("stream read grid %d: %.1f GB/s\n", grid, 5.0 * bytes / (ms * 1e-3) / 1e9);
  }
  // 3. 8 concurrent streams, 512 MiB each
  hipStream_t ws[8]; for (int i = 0; i < 8; ++i) CK(hipStreamCreateWithFlags(&ws[i], hipStreamNonBlocking));
  CK(hipDeviceSynchronize());
  for (int rep = 0; rep < 3; ++rep) {
    auto t0 = clk::now();
    for (int i = 0; i < 8; ++i) hipLaunchKernelGGL(stream_sum, dim3(512), dim3(256), 0, ws[i], a + (size_t)i * (bytes / 16 / 8), bytes / 16 / 8, out);
    CK(hipDeviceSynchronize());
    double t = us(t0, clk::now());
    printf("8 streams x 512MiB: %.1f us -> %.1f GB/s\n", t, bytes / (t * 1e-6) / 1e9);
  }
  // 4. realtime tick
  unsigned long long* rt; CK(hipMalloc(&rt, 16));
  hipLaunchKernelGGL(realtime_kernel, dim3(1), dim3(64), 0, s, rt, 1000);
  unsigned long long hrt[2]; CK(hipMemcpy(hrt, rt, 16, hipMemcpyDeviceToHost));
  auto w0 = clk::now();
  hipLaunchKernelGGL(realtime_kernel, dim3(1), dim3(64), 0, s, rt, 5000); CK(hipStreamSynchronize(s));
  printf("realtime spin 5000us took host %.1f us; ticks %llu memtime %llu\n", us(w0, clk::now()), hrt[0], hrt[1]);
  return 0;
}
