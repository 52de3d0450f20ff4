// Probe: what an LDS-DMA instruction costs the issuing wave when it runs beside an MFMA
// stream at one wave per SIMD (the c5 lsqp4 kernel's situation: profiles/r02_c5_sq_counters.txt).
// Every CU runs one 4-wave workgroup; each wave issues, per loop step, 16 independent
// v_mfma_f32_16x16x32_bf16 (4 accumulators) with D LDS-DMA pieces (1 KiB each) spread among
// them, streaming a large buffer from HBM (outstanding loads bounded like the kernel's ring).
// Forms of the DMA:
//   1 global_load_lds_dwordx4 v_off, s_base          (saddr + 32-bit lane offset; lsqp4's form)
//   2 global_load_lds_dwordx4 v_addr64, off           (64-bit lane address)
//   3 buffer_load_dwordx4 v_off, s_rsrc, 0 offen lds   (descriptor + lane offset)
// (a fourth form, buffer_load ... lds with an ADD_TID descriptor and no lane address, faulted
// the GPU on the first run: the descriptor bits assumed for it are not gfx950's; removed)
// Each form streams from a buffer that lives in HBM (4 GiB), the Infinity Cache (128 MiB) or
// L2 (16 MiB over 8 XCDs): the per-CU ingest rate tells a per-CU LDS-DMA limit from HBM's.
// Prints the time per step and the cost per DMA over the MFMA-only stream.
//   hipcc --offload-arch=gfx950 -O3 -o probe_dma_issue tools/probe_dma_issue.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_) { std::printf("FAIL %s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } \
  } while (0)

template <int FORM, int D, bool MF = true, int VM = 24>
__global__ void __launch_bounds__(256, 1) probe(const uint8_t* __restrict__ buf, size_t bytes, int steps, float* out) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[4][16384];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ldsb = __builtin_amdgcn_readfirstlane(uint32_t(uintptr_t(&ring[w][0])));
  // each wave streams its own region of the buffer, 1 KiB per DMA
  const size_t per_wave = bytes / (gridDim.x * 4) / 1024 * 1024;
  const uint64_t bu = uint64_t(uintptr_t(buf + (size_t(blockIdx.x) * 4 + w) * per_wave));
  // wave-uniform in SGPRs; the halves widened as UNSIGNED (readfirstlane returns int)
  const uint64_t lo = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(bu)));
  const uint64_t hi = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(bu >> 32)));
  const uint8_t* base = reinterpret_cast<const uint8_t*>(uintptr_t(lo | hi << 32));
  auto rsrc0 = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
  bf16x8 a = __builtin_bit_cast(bf16x8, make_uint4(lane, lane + 1, lane + 2, lane + 3));
  bf16x8 b = __builtin_bit_cast(bf16x8, make_uint4(lane * 3, 7, 9, lane));
  f32x4 acc[4] = {};
  size_t off = 0;
  int piece = 0;
  for (int st = 0; st < steps; ++st) {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if (MF) acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m & 3], 0, 0, 0);
      if (D > 0 && (m % (16 / (D > 16 ? 16 : D))) == 0) {
#pragma unroll
        for (int d = 0; d < (D > 16 ? D / 16 : 1); ++d) {
          const uint32_t lds = ldsb + uint32_t(piece & 15) * 1024;
          const uint32_t voff = uint32_t(off) + uint32_t(lane) * 16;
          if (FORM == 1) {
            asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(base), "s"(lds)
                         : "memory");
          } else if (FORM == 2) {
            const uint8_t* p = base + voff;
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(p), "s"(lds) : "memory");
          } else {
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %0, 0 offen lds" ::"s"(rsrc0), "s"(lds),
                         "v"(voff)
                         : "memory");
          }
          off += 1024;
          if (off + 1024 > per_wave) off = 0;
          ++piece;
          // bound the loads in flight (the kernel keeps ~20-34): wait for all but VM
          if ((piece & 7) == 0) {
            if (VM == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (VM == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            else if (VM == 40) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
            else if (VM == 54) asm volatile("s_waitcnt vmcnt(54)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
          }
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  s += float(ring[w][lane * 4]);
  if (s == 1234.5f) out[threadIdx.x] = s;  // never true; keeps the work alive
}

template <int FORM, int D, bool MF = true, int VM = 24>
double run(const uint8_t* buf, size_t bytes, int steps, float* out, int grid) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  probe<FORM, D, MF, VM><<<grid, 256>>>(buf, bytes, 4, out);  // warm-up
  CK(hipDeviceSynchronize());
  double best = 1e30;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(a));
    probe<FORM, D, MF, VM><<<grid, 256>>>(buf, bytes, steps, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return best;
}

int main() {
  const size_t big = size_t(4) << 30;
  uint8_t* buf;
  float* out;
  CK(hipMalloc(&buf, big));
  CK(hipMemset(buf, 1, big));
  CK(hipMalloc(&out, 4096));
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int steps = 4000, grid = cus;
  const double t0 = run<1, 0>(buf, big, steps, out, grid);
  std::printf("mfma only: %.3f ms, %.1f ns per 16-MFMA step\n", t0, t0 * 1e6 / steps);
  struct R { const char* name; double (*f)(const uint8_t*, size_t, int, float*, int); int d; bool mf; };
  const R rs[] = {
      {"glds saddr   D=2 ", run<1, 2>, 2, true},   {"glds saddr   D=4 ", run<1, 4>, 4, true},
      {"glds saddr   D=8 ", run<1, 8>, 8, true},   {"glds saddr   D=16", run<1, 16>, 16, true},
      {"glds vaddr64 D=4 ", run<2, 4>, 4, true},   {"buf offen    D=4 ", run<3, 4>, 4, true},
      {"glds no-MFMA D=16", run<1, 16, false>, 16, false},
  };
  const struct { const char* where; size_t bytes; } places[] = {{"HBM 4 GiB", big}};
  for (const auto& pl : places) {
    std::printf("-- buffer %s (%.0f KiB per wave)\n", pl.where, double(pl.bytes) / (grid * 4) / 1024);
    for (const R& r : rs) {
      const double t = r.f(buf, pl.bytes, steps, out, grid);
      const double per_step_ns = t * 1e6 / steps, extra_ns = (t - t0) * 1e6 / steps / r.d;
      const double gbs = double(steps) * r.d * 1024.0 * grid * 4 / (t * 1e-3) / 1e9;
      std::printf("%s %.3f ms  %.1f ns/step  +%.1f ns per DMA over MFMA-only  %.0f GB/s chip = %.1f GB/s per CU\n",
                  r.name, t, per_step_ns, extra_ns, gbs, gbs / grid);
    }
  }
  // loads in flight: the wave waits for all but VM of its DMAs every 8 (HBM buffer)
  const R vs[] = {{"glds saddr   D=8  vm8 ", run<1, 8, true, 8>, 8, true},
                  {"glds saddr   D=8  vm16", run<1, 8, true, 16>, 8, true},
                  {"glds saddr   D=8  vm24", run<1, 8, true, 24>, 8, true},
                  {"glds saddr   D=8  vm40", run<1, 8, true, 40>, 8, true},
                  {"glds saddr   D=8  vm54", run<1, 8, true, 54>, 8, true},
                  {"glds no-MFMA D=16 vm54", run<1, 16, false, 54>, 16, false}};
  std::printf("-- loads in flight, buffer HBM 4 GiB\n");
  for (const R& r : vs) {
    const double t = r.f(buf, big, steps, out, grid);
    const double gbs = double(steps) * r.d * 1024.0 * grid * 4 / (t * 1e-3) / 1e9;
    std::printf("%s %.3f ms  %.0f GB/s chip = %.1f GB/s per CU\n", r.name, t, gbs, gbs / grid);
  }
  std::printf("ok\n");
  return 0;
}
