// Host cost of hipLaunchKernelGGL against the kernel-argument size (round 6: a server's
// host-launched least-squares task spends 4-12 us inside the launch call, tools/gpu_r06hl.sh;
// LsqBatch is 3656 B).  For each size: 2000 launches of an empty kernel on one stream, the
// mean host time of the launch call alone, and the launch-to-start latency on an idle queue
// (the launch timed on the host, the kernel's start by s_memrealtime against a host/device
// clock pair taken first).
//   hipcc --offload-arch=gfx950 -O2 -o tools/bin/probe_launch tools/probe_launch.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

template <int N>
struct Args {
  unsigned long long* out;
  unsigned char pad[N];
};

template <int N>
__global__ void empty_kernel(Args<N> a) {
  if (threadIdx.x == 0 && blockIdx.x == 0) a.out[0] = __builtin_amdgcn_s_memrealtime() + a.pad[N - 1];
}

using Clk = std::chrono::steady_clock;

template <int N>
int probe(hipStream_t s, unsigned long long* out, const char* label) {
  Args<N> a{};
  a.out = out;
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(empty_kernel<N>, dim3(1), dim3(64), 0, s, a);
  CK(hipStreamSynchronize(s));
  // back-to-back launches: host time per call
  const int K = 2000;
  double tot = 0;
  for (int i = 0; i < K; ++i) {
    const auto t0 = Clk::now();
    hipLaunchKernelGGL(empty_kernel<N>, dim3(1), dim3(64), 0, s, a);
    tot += std::chrono::duration<double, std::micro>(Clk::now() - t0).count();
    if (i % 64 == 63) CK(hipStreamSynchronize(s));
  }
  CK(hipStreamSynchronize(s));
  // one launch onto an idle queue: call time, and host call -> synchronize return
  std::vector<double> call, rt;
  for (int i = 0; i < 300; ++i) {
    const auto t0 = Clk::now();
    hipLaunchKernelGGL(empty_kernel<N>, dim3(1), dim3(64), 0, s, a);
    const auto t1 = Clk::now();
    CK(hipStreamSynchronize(s));
    const auto t2 = Clk::now();
    call.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    rt.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
  }
  std::sort(call.begin(), call.end());
  std::sort(rt.begin(), rt.end());
  std::printf("%-10s kernarg %5zu B: back-to-back launch call %6.2f us; idle queue: call p50 %6.2f us, launch -> sync "
              "return p50 %6.2f us\n", label, sizeof(Args<N>), tot / K, call[call.size() / 2], rt[rt.size() / 2]);
  return 0;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned long long* out;
  CK(hipMalloc(&out, 64));
  if (probe<8>(s, out, "tiny")) return 1;
  if (probe<256>(s, out, "256")) return 1;
  if (probe<1024>(s, out, "1k")) return 1;
  if (probe<2048>(s, out, "2k")) return 1;
  if (probe<3648>(s, out, "LsqBatch")) return 1;
  if (probe<8>(s, out, "tiny")) return 1;
  return 0;
}
