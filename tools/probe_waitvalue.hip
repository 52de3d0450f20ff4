// Probe: can a worker stream be pre-armed to wait on a doorbell word that another party
// (host thread here; another process's exchange kernel in the product) rings?
//   hipStreamWaitValue64(stream, word, seq, hipStreamWaitValueGte) -> task kernel -> flag
// For each memory kind of the doorbell word (hipHostMalloc coherent, hipHostRegister'ed
// malloc, device memory written by a kernel) it measures ring -> task-flag-visible latency
// against a host poll + hipLaunchKernel baseline.  Not product code; feeds DESIGN.md §5.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include <algorithm>

#define CK(x)                                                                                       \
  do {                                                                                              \
    hipError_t e = (x);                                                                             \
    if (e != hipSuccess) {                                                                          \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);                  \
      return 1;                                                                                     \
    }                                                                                               \
  } while (0)
using clk = std::chrono::steady_clock;

__global__ void flag_kernel(unsigned long long* flag, unsigned long long v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
__global__ void ring_kernel(unsigned long long* door, unsigned long long v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(door, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? -1 : v[v.size() / 2];
}

int main() {
  CK(hipSetDevice(0));
  unsigned long long* flag;
  CK(hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const int N = 200;

  // baseline: host sees a host word change, then launches the task kernel
  {
    volatile unsigned long long* door;
    CK(hipHostMalloc((void**)&door, 64, hipHostMallocCoherent | hipHostMallocMapped));
    std::vector<double> lat;
    *flag = 0;
    *door = 0;
    for (int k = 1; k <= N; ++k) {
      std::thread ringer([&]() {
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        __atomic_store_n((unsigned long long*)door, (unsigned long long)k, __ATOMIC_RELEASE);
      });
      while (__atomic_load_n((unsigned long long*)door, __ATOMIC_ACQUIRE) < (unsigned long long)k) {
      }
      const auto t0 = clk::now();
      hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, flag, (unsigned long long)k);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) < (unsigned long long)k) {
      }
      lat.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
      ringer.join();
    }
    CK(hipStreamSynchronize(s));
    printf("host-poll + launch: ring->flag median %.2f us\n", median(lat));
  }

  // pre-armed stream wait on three kinds of doorbell memory
  for (int kind = 0; kind < 3; ++kind) {
    unsigned long long* door_host = nullptr;
    unsigned long long* door_dev = nullptr;
    void* raw = nullptr;
    const char* name = kind == 0 ? "hipHostMalloc coherent" : kind == 1 ? "hipHostRegister'ed malloc" : "device memory";
    if (kind == 0) {
      CK(hipHostMalloc((void**)&door_host, 64, hipHostMallocCoherent | hipHostMallocMapped));
      door_dev = door_host;
    } else if (kind == 1) {
      raw = aligned_alloc(4096, 4096);
      door_host = (unsigned long long*)raw;
      CK(hipHostRegister(raw, 4096, hipHostRegisterMapped));
      CK(hipHostGetDevicePointer((void**)&door_dev, raw, 0));
    } else {
      CK(hipMalloc((void**)&door_dev, 64));
    }
    if (door_host) *door_host = 0;
    else CK(hipMemset(door_dev, 0, 64));
    CK(hipDeviceSynchronize());
    *flag = 0;
    std::vector<double> lat;
    bool ok = true;
    for (int k = 1; k <= N && ok; ++k) {
      hipError_t e = hipStreamWaitValue64(s, door_dev, (uint64_t)k, hipStreamWaitValueGte, ~0ull);
      if (e != hipSuccess) {
        printf("%s: hipStreamWaitValue64 failed: %s\n", name, hipGetErrorString(e));
        ok = false;
        break;
      }
      hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, flag, (unsigned long long)k);
      std::this_thread::sleep_for(std::chrono::microseconds(300));
      if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) >= (unsigned long long)k) {
        printf("%s: the task ran before the ring (wait did not hold)\n", name);
        ok = false;
        break;
      }
      const auto t0 = clk::now();
      if (door_host) __atomic_store_n(door_host, (unsigned long long)k, __ATOMIC_RELEASE);
      else hipLaunchKernelGGL(ring_kernel, dim3(1), dim3(64), 0, s2, door_dev, (unsigned long long)k);
      const auto tw = clk::now();
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) < (unsigned long long)k) {
        if (std::chrono::duration<double>(clk::now() - tw).count() > 2.0) {
          printf("%s: task never ran after the ring (timeout)\n", name);
          ok = false;
          break;
        }
      }
      lat.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    }
    if (!ok) {
      // release the armed wait so the stream drains
      if (door_host) __atomic_store_n(door_host, ~0ull >> 1, __ATOMIC_RELEASE);
      else hipLaunchKernelGGL(ring_kernel, dim3(1), dim3(64), 0, s2, door_dev, ~0ull >> 1);
    }
    CK(hipStreamSynchronize(s));
    CK(hipStreamSynchronize(s2));
    if (ok) printf("%s: pre-armed wait ring->flag median %.2f us (%zu samples)\n", name, median(lat), lat.size());
    if (kind == 1) {
      CK(hipHostUnregister(raw));
      free(raw);
    }
  }
  return 0;
}
