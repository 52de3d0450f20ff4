// Which CU does each bit of a stream's CU mask (hipExtStreamCreateWithCUMask) stand for on this
// part?  For a mask with one bit cleared, a kernel of 2048 one-wave workgroups (each spinning
// ~20 us so that every enabled CU takes several) records the (XCC, SE, CU) it ran on; the CU
// that no longer appears is the bit's.  Also the number of distinct CUs under the full mask and
// under a mask with one bit per 32-bit word cleared.  Measurement tool (round 6): the coordinator
// CU reservation at N > 1 needs one reserved CU per XCD.
//   hipcc --offload-arch=gfx950 -O2 -o tools/bin/probe_cumask tools/probe_cumask.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

__global__ void where_kernel(unsigned* out, unsigned long long spin) {
  if (threadIdx.x) return;
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(1);
  out[blockIdx.x] = ((xcc & 0xF) << 16) | (hw & 0xFFFF);
}

using Cu = std::tuple<unsigned, unsigned, unsigned, unsigned>;  // xcc, se, sh, cu
static Cu decode(unsigned v) {
  const unsigned hw = v & 0xFFFF;
  return {v >> 16, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15};
}

static int run(const std::vector<uint32_t>& mask, std::set<Cu>* used) {
  hipStream_t s;
  CK(hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()));
  const int grid = 2048;
  unsigned* d;
  CK(hipMalloc(&d, grid * sizeof(unsigned)));
  hipLaunchKernelGGL(where_kernel, dim3(grid), dim3(64), 0, s, d, 2000ull);  // 20 us at 100 MHz
  CK(hipStreamSynchronize(s));
  std::vector<unsigned> h(grid);
  CK(hipMemcpy(h.data(), d, grid * sizeof(unsigned), hipMemcpyDeviceToHost));
  for (unsigned v : h) used->insert(decode(v));
  CK(hipFree(d));
  CK(hipStreamDestroy(s));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const size_t words = size_t((cus + 31) / 32);
  std::vector<uint32_t> full(words, 0xFFFFFFFFu);
  if (cus % 32) full.back() = (1u << (cus % 32)) - 1u;
  std::set<Cu> all;
  if (run(full, &all)) return 1;
  std::printf("%s: %d CUs, full mask -> %zu distinct (xcc, se, sh, cu)\n", p.gcnArchName, cus, all.size());
  std::set<unsigned> xccs;
  for (const auto& c : all) xccs.insert(std::get<0>(c));
  std::printf("XCCs seen: %zu\n", xccs.size());
  const int bits[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 15, 16, 31, 32, 33, 63, 64, 255};
  for (int b : bits) {
    if (b >= cus) continue;
    std::vector<uint32_t> m = full;
    m[size_t(b / 32)] &= ~(1u << (b % 32));
    std::set<Cu> u;
    if (run(m, &u)) return 1;
    std::printf("bit %3d cleared: %zu CUs used; missing:", b, u.size());
    for (const auto& c : all)
      if (!u.count(c)) std::printf(" (xcc %u se %u sh %u cu %u)", std::get<0>(c), std::get<1>(c), std::get<2>(c), std::get<3>(c));
    std::printf("\n");
  }
  // one bit per 32-bit word cleared (bits 0, 32, 64, ...)
  std::vector<uint32_t> m = full;
  for (size_t w = 0; w < words; ++w) m[w] &= ~1u;
  std::set<Cu> u;
  if (run(m, &u)) return 1;
  std::set<unsigned> per;
  std::printf("bits 0, 32, 64, ... cleared: %zu CUs used; missing:", u.size());
  for (const auto& c : all)
    if (!u.count(c)) std::printf(" (xcc %u se %u cu %u)", std::get<0>(c), std::get<1>(c), std::get<3>(c));
  std::printf("\n");
  // bits 0..7 cleared
  m = full;
  m[0] &= ~0xFFu;
  u.clear();
  if (run(m, &u)) return 1;
  std::printf("bits 0-7 cleared: %zu CUs used; missing:", u.size());
  for (const auto& c : all)
    if (!u.count(c)) std::printf(" (xcc %u se %u cu %u)", std::get<0>(c), std::get<1>(c), std::get<3>(c));
  std::printf("\n");
  return 0;
}
