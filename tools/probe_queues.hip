// Probe: do kernels on K HIP streams run concurrently?  Launches one 20 ms spin kernel
// (1 workgroup, s_memrealtime) per stream and times the whole set on the host.  Streams are
// plain (hipStreamCreateWithFlags) or CU-masked with every CU enabled
// (hipExtStreamCreateWithCUMask), which asks the runtime for a queue of their own.
// Not product code; the result decides how the transport creates worker streams.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void spin(unsigned long long ticks) {
  if (threadIdx.x) return;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}

int main() {
  int khz = 0;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  printf("wallclock rate %d kHz\n", khz);
  const unsigned long long ticks = (unsigned long long)(0.020 * khz * 1e3);
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, 0, 1000ull);
  (void)hipDeviceSynchronize();
  for (int mode = 0; mode < 2; ++mode) {
    for (int k : {2, 4, 8, 12, 16}) {
      std::vector<hipStream_t> s(k);
      for (auto& x : s) {
        if (mode == 0) {
          (void)hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
        } else {
          std::vector<uint32_t> mask(8, 0xFFFFFFFFu);
          (void)hipExtStreamCreateWithCUMask(&x, (uint32_t)mask.size(), mask.data());
        }
      }
      for (auto& x : s) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, x, 1000ull);
      (void)hipDeviceSynchronize();
      auto t0 = std::chrono::steady_clock::now();
      for (auto& x : s) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, x, ticks);
      (void)hipDeviceSynchronize();
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      printf("%s streams=%2d  20ms spins took %.1f ms  (%.1f x serial)\n", mode ? "cumask" : "plain ", k, ms, ms / 20.0);
      for (auto& x : s) (void)hipStreamDestroy(x);
    }
  }
  return 0;
}
