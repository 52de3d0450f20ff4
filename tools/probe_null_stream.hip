// Probe: which stream kinds make the legacy NULL stream wait for their work, and which get
// an HSA queue of their own.  For each kind: the stream's flags; the host time of a
// NULL-stream hipMemcpy (device -> host, 8 bytes) issued while a 50 ms one-wave spin runs on
// that stream (~0 ms: the NULL stream does not wait for it; ~50 ms: it does); and 8 streams of
// the kind each running a 20 ms spin at once (20 ms: a queue each; 40+: shared queues).
// Not product code: the result decides how a delayed worker may sleep on the device.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

__global__ void spin(unsigned long long ticks) {
  if (threadIdx.x) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static hipStream_t make(int kind) {
  hipStream_t s = nullptr;
  std::vector<uint32_t> mask(8, 0xFFFFFFFFu);
  if (kind == 0) (void)hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data());
  if (kind == 1) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (kind == 2) (void)hipStreamCreateWithFlags(&s, hipStreamDefault);
  if (kind == 3) {
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    (void)hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi);
  }
  return s;
}

int main() {
  const char* names[] = {"cu-mask", "plain non-blocking", "plain blocking", "priority(high) non-blocking"};
  int khz = 0;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  const unsigned long long ms = (unsigned long long)khz;  // ticks per ms
  void* dbuf = nullptr;
  (void)hipMalloc(&dbuf, 64);
  unsigned long long host = 0;
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, 0, 10ull);
  (void)hipDeviceSynchronize();
  for (int kind = 0; kind < 4; ++kind) {
    hipStream_t s = make(kind);
    unsigned flags = 99;
    (void)hipStreamGetFlags(s, &flags);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 50 * ms);
    const double t0 = now_ms();
    (void)hipMemcpy(&host, dbuf, 8, hipMemcpyDeviceToHost);  // NULL stream
    const double waited = now_ms() - t0;
    (void)hipDeviceSynchronize();
    std::vector<hipStream_t> v(8);
    for (auto& x : v) x = make(kind);
    for (auto& x : v) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, x, 1ull);
    (void)hipDeviceSynchronize();
    const double t1 = now_ms();
    for (auto& x : v) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, x, 20 * ms);
    (void)hipDeviceSynchronize();
    const double conc = now_ms() - t1;
    std::printf("%-28s flags %u  NULL-stream memcpy behind a 50 ms spin: %.1f ms  8 x 20 ms spins: %.1f ms\n",
                names[kind], flags, waited, conc);
    std::fflush(stdout);
  }
  return 0;
}
