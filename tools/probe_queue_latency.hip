// Probe: launch -> start latency of a tiny kernel on one of Q idle HSA queues, as a
// function of how many queues the process holds (CU-masked streams, each its own queue),
// with and without B queues kept busy by a spinning kernel (a sleeping straggler).
// The kernel writes s_memrealtime into host-pinned memory; the host polls it.  Reports
// median / p99 / max of (host sees the word - host launch call start) over many launches
// on randomly chosen queues.  Not product code: the result decides how many queues the
// transport may hold.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__global__ void stamp(volatile unsigned long long* out, unsigned long long tag) {
  if (threadIdx.x) return;
  __atomic_store_n(const_cast<unsigned long long*>(out), tag, __ATOMIC_RELEASE);
}

__global__ void spin(unsigned long long ticks) {
  if (threadIdx.x) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 400;
  int khz = 0;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  unsigned long long* word = nullptr;
  (void)hipHostMalloc(reinterpret_cast<void**>(&word), 64, hipHostMallocCoherent);
  *word = 0;
  std::mt19937 rng(7);
  unsigned long long tag = 0;
  // queues are only ever added (never destroyed: a destroy is not what the transport does,
  // and the first version of this probe hung in one), so the process holds q queues at step q
  std::vector<hipStream_t> s;
  std::vector<uint32_t> mask(8, 0xFFFFFFFFu);
  for (int q : {4, 8, 12, 16, 20, 24, 32}) {
    const double tc = now_us();
    while (int(s.size()) < q) {
      hipStream_t x = nullptr;
      if (hipExtStreamCreateWithCUMask(&x, uint32_t(mask.size()), mask.data()) != hipSuccess) {
        std::printf("stream create failed at %zu\n", s.size());
        return 1;
      }
      hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, x, word, ++tag);
      s.push_back(x);
    }
    (void)hipDeviceSynchronize();
    std::printf("-- %d queues (created in %.1f ms)\n", q, (now_us() - tc) / 1e3);
    std::fflush(stdout);
    for (int busy : {0, 2}) {
      std::vector<double> lat;
      double t_end_busy = 0;
      for (int it = 0; it < iters; ++it) {
        // the first `busy` queues hold a 30 ms spin, renewed when it ends
        if (busy && now_us() > t_end_busy) {
          for (int b = 0; b < busy; ++b)
            hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[size_t(b)], (unsigned long long)(0.030 * khz * 1e3));
          t_end_busy = now_us() + 30000;
        }
        const int k = busy + int(rng() % unsigned(q - busy));
        const unsigned long long t = ++tag;
        const double t0 = now_us();
        hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, s[size_t(k)], word, t);
        while (__atomic_load_n(word, __ATOMIC_ACQUIRE) != t) {
          if (now_us() - t0 > 2e6) {
            std::printf("stuck: queues %d busy %d iteration %d\n", q, busy, it);
            return 1;
          }
        }
        lat.push_back(now_us() - t0);
        const double pause = 200 + double(rng() % 800);  // idle 0.2-1 ms between launches
        const double tp = now_us();
        while (now_us() - tp < pause) {
        }
      }
      (void)hipDeviceSynchronize();
      std::sort(lat.begin(), lat.end());
      int over1ms = 0;
      for (double v : lat) over1ms += v > 1000;
      std::printf("queues=%2d busy=%d  launch->visible us: median %.1f p99 %.1f max %.1f  (>1 ms: %d of %zu)\n", q, busy,
                  lat[lat.size() / 2], lat[lat.size() * 99 / 100], lat.back(), over1ms, lat.size());
      std::fflush(stdout);
    }
  }
  return 0;
}
