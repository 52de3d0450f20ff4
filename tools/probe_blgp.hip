// Does v_mfma_f32_16x16x32_bf16's BLGP field (B-matrix lane-group pattern) broadcast on gfx950?
// BLGP 1: lanes 32-63 take the B operand of lanes 0-31; BLGP 2: lanes 0-31 take that of lanes
// 32-63.  lsqp4's phase 2 reads each A element twice (k 0-15 the hi residual, k 16-31 the lo
// residual of the SAME rows: lanes 32-63 hold a copy of lanes 0-31's B operand); with the
// broadcast, one transposed read could carry two column tiles.
// One wave: random A, B in bf16; D = A x B with BLGP 0 on a B whose upper half copies the lower
// (reference) against BLGP 1 on a B whose upper half is garbage, and BLGP 2 on one whose lower half
// is garbage.  Prints the max |difference| (0 = the broadcast works, bit for bit).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/probe_blgp tools/probe_blgp.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// out[l * 32 + 4 * v + r]: v = 0 the reference (blgp 0 on the full copy), v = 1..7 blgp v on the
// B with garbage in lanes 32-63 (the lower half valid); out[l * 32 + 16 + ...] the same on the B
// with garbage in lanes 0-31 (the upper half valid)
template <int BL>
__device__ void one(const bf16x8& av, const bf16x8& bl, const bf16x8& bh, float* out, int l) {
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  const f32x4 d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bl, z, 0, 0, BL);
  const f32x4 d2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bh, z, 0, 0, BL);
  for (int r = 0; r < 4; ++r) {
    out[l * 64 + 8 * BL + r] = d1[r];
    out[l * 64 + 8 * BL + 4 + r] = d2[r];
  }
}

__global__ void __launch_bounds__(64) probe(const unsigned short* a, const unsigned short* b, float* out) {
  const int l = threadIdx.x;
  bf16x8 av, bv, bl, bh;
  for (int j = 0; j < 8; ++j) {
    av[j] = __builtin_bit_cast(__bf16, a[l * 8 + j]);
    const unsigned short lo = b[(l & 31) * 8 + j];              // lanes l and l + 32 alike
    bv[j] = __builtin_bit_cast(__bf16, lo);
    bl[j] = __builtin_bit_cast(__bf16, l < 32 ? lo : (unsigned short)0x7f7f);   // upper half garbage
    bh[j] = __builtin_bit_cast(__bf16, l >= 32 ? lo : (unsigned short)0x7f7f);  // lower half garbage
  }
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  const f32x4 ref = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, z, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 64 + r] = ref[r];
  one<1>(av, bl, bh, out, l);
  one<2>(av, bl, bh, out, l);
  one<3>(av, bl, bh, out, l);
  one<4>(av, bl, bh, out, l);
  one<5>(av, bl, bh, out, l);
  one<6>(av, bl, bh, out, l);
  one<7>(av, bl, bh, out, l);
}

int main() {
  unsigned short ha[512], hb[512];
  srand(7);
  for (int i = 0; i < 512; ++i) {
    const float f = float(rand()) / RAND_MAX * 2.f - 1.f;
    unsigned u;
    __builtin_memcpy(&u, &f, 4);
    ha[i] = (unsigned short)(u >> 16);
    const float g = float(rand()) / RAND_MAX * 2.f - 1.f;
    __builtin_memcpy(&u, &g, 4);
    hb[i] = (unsigned short)(u >> 16);
  }
  unsigned short *da, *db;
  float* dout;
  hipMalloc(&da, sizeof(ha));
  hipMalloc(&db, sizeof(hb));
  hipMalloc(&dout, 64 * 64 * sizeof(float));
  hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
  hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dout);
  static float h[64 * 64];
  if (hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) {
    std::printf("launch failed\n");
    return 1;
  }
  for (int bl = 1; bl < 8; ++bl) {
    double m1 = 0, m2 = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        m1 = fmax(m1, fabs(h[l * 64 + 8 * bl + r] - h[l * 64 + r]));
        m2 = fmax(m2, fabs(h[l * 64 + 8 * bl + 4 + r] - h[l * 64 + r]));
      }
    std::printf("blgp %d: lower half valid max |D - ref| = %g | upper half valid max |D - ref| = %g\n", bl, m1, m2);
  }
  return 0;
}
