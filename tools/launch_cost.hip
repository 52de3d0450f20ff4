// Launch round trip on the coordinator's critical path, by kernel-argument size: the host
// launches a kernel whose one workgroup writes a host-pinned completion word, and spins on
// it before the next launch (c1's epoch without the compute).  Also the back-to-back host
// cost of hipLaunchKernel alone, and a ping-pong with a resident kernel (the floor a
// pre-armed launch could reach).  tools/gpu_r03zi.sh; profiles/r03_launch_cost.txt.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

template <int BYTES>
struct Args {
  unsigned long long* flag;
  unsigned long long seq;
  unsigned char pad[BYTES - 16];
};

template <int BYTES>
__global__ void publish(Args<BYTES> a) {
  if (threadIdx.x == 0 && blockIdx.x == 0)
    __hip_atomic_store(a.flag, a.seq + a.pad[7], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// resident: waits for go == k (host-pinned), answers done = k, n times; bounded spin
__global__ void pingpong(const unsigned long long* go, unsigned long long* done, int n, unsigned* err) {
  if (threadIdx.x != 0) return;
  for (int k = 1; k <= n; ++k) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < (unsigned long long)k) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 500000000ull) {  // 5 s at 100 MHz
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
    }
    __hip_atomic_store(done, (unsigned long long)k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

using Clock = std::chrono::steady_clock;

template <int BYTES>
void round_trip(hipStream_t s, unsigned long long* flag, int n) {
  Args<BYTES> a{};
  a.flag = flag;
  for (int k = 0; k < 200; ++k) {  // warm
    a.seq = 100000000ull + k;
    hipLaunchKernelGGL(publish<BYTES>, dim3(1), dim3(64), 0, s, a);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != a.seq) {}
  }
  const auto t0 = Clock::now();
  double launch_us = 0;
  for (int k = 0; k < n; ++k) {
    a.seq = 1000 + k;
    const auto l0 = Clock::now();
    hipLaunchKernelGGL(publish<BYTES>, dim3(1), dim3(64), 0, s, a);
    launch_us += std::chrono::duration<double, std::micro>(Clock::now() - l0).count();
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != a.seq) {}
  }
  const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count() / n;
  CK(hipStreamSynchronize(s));
  // back to back, no waiting
  const auto b0 = Clock::now();
  for (int k = 0; k < n; ++k) {
    a.seq = 5000000 + k;
    hipLaunchKernelGGL(publish<BYTES>, dim3(1), dim3(64), 0, s, a);
  }
  const double b2b = std::chrono::duration<double, std::micro>(Clock::now() - b0).count() / n;
  CK(hipStreamSynchronize(s));
  std::printf("kernarg %5d B: launch+complete+observe %.2f us (hipLaunchKernel %.2f us of it); back-to-back launch %.2f us\n",
              BYTES, us, launch_us / n, b2b);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned long long *flag, *go, *done;
  unsigned* err;
  CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocCoherent));
  CK(hipHostMalloc(reinterpret_cast<void**>(&go), 64, hipHostMallocCoherent));
  CK(hipHostMalloc(reinterpret_cast<void**>(&done), 64, hipHostMallocCoherent));
  CK(hipHostMalloc(reinterpret_cast<void**>(&err), 64, hipHostMallocCoherent));
  *flag = *go = *done = 0;
  *err = 0;
  const int n = 5000;
  round_trip<64>(s, flag, n);
  round_trip<1024>(s, flag, n);
  round_trip<2048>(s, flag, n);
  round_trip<3456>(s, flag, n);
  // ping-pong with a resident kernel
  hipLaunchKernelGGL(pingpong, dim3(1), dim3(64), 0, s, go, done, n + 100, err);
  for (int k = 1; k <= 100; ++k) {
    __atomic_store_n(go, (unsigned long long)k, __ATOMIC_RELEASE);
    while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != (unsigned long long)k && !*(volatile unsigned*)err) {}
  }
  const auto t0 = Clock::now();
  for (int k = 101; k <= n + 100; ++k) {
    __atomic_store_n(go, (unsigned long long)k, __ATOMIC_RELEASE);
    while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != (unsigned long long)k && !*(volatile unsigned*)err) {}
  }
  const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count() / n;
  CK(hipStreamSynchronize(s));
  std::printf("resident kernel ping-pong (host go word -> device -> host done word): %.2f us, err %u\n", us, *err);
  return 0;
}
