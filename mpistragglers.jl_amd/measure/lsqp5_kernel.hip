// Single-pass batched least squares by iterate halves, one wave per SIMD, phase 2 as
// 32x32x16 MFMAs (BASELINE configs[4], "c5"):
//     G_i = A_i^T (A_i X - B_i)      A_i rows x cols bf16, X cols x 64 bf16, B_i rows x 64 bf16
// in the reference's compute slot (examples/iterative_example.jl:74 sleeps there), A read
// from HBM once.  lsqp4_kernel.hip's scheme (pairs of workgroups on one XCD, member h owning
// iterates 32h .. 32h + 31; 4 waves, one per SIMD, wave w owning columns 512 w .. 512 w + 511;
// a 2-slot strip ring per wave; phase 1 split-K over the waves; one barrier per block), with
// phase 2 re-cut (round 4, VERDICT r03 item 5):
//
//   phase 2   G_w^T[32 its][512 cols] += R^T[32 its][16 rows] A[16 rows][512 cols], as 16
//             column tiles of 32 x 32 (f32x16 each, 256 AGPRs): per tile ONE transposed
//             B operand (A[rows 8h .. 8h + 7][32 columns], two ds_read_b64_tr_b16) and TWO
//             32x32x16 MFMAs, one with the bf16 hi part of R and one with the lo part.
//
// lsqp4 ran phase 2 as 16x16x32 MFMAs with k 0-15 the hi and k 16-31 the lo residual of the
// SAME 16 rows: every A row was read twice from LDS and every tile took 2 MFMAs per 16
// columns.  Here each A element is read once (32 transposed reads per block instead of 64),
// the MFMA count halves (32 instead of 64, the same MFMA cycles), and each 32-cycle MFMA hides
// more of the wave's other issue.  The reduce moves R into the 32x32x16 A-operand layout with
// one v_permlane16_swap per register pair (lsqp4: a permlane32 and a permlane16 swap).  The
// strip swizzle is re-searched for the new read (sw below; tools/lsqp4_swizzle.py --p5).
//
// MFMA maps (cdna_hip_programming.md §3): 16x16x32 bf16 (phase 1): A[m=i][k=8g+j],
// B[k=8g+j][n=i], C/D[m=4g+r][n=i]; lane l: i = l & 15, g = l >> 4.  32x32x16 bf16 (phase 2):
// A[m=l&31][k=8h+j], B[k=8h+j][n=l&31], C/D[m=(r&3)+8(r>>2)+4h][n=l&31]; h = l >> 5.
#include <hip/hip_runtime.h>

#include "device_common.hpp"
#include "kernels.hpp"
#include "mpiasyncpools.h"


namespace mpa {
namespace {

using namespace dev;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int K = kLsqbIterates;      // 64 iterates
constexpr int QW = 4;                 // waves per workgroup, one per SIMD
constexpr int QT = QW * 64;           // threads
constexpr int PRB = 16;               // rows per block
constexpr int QKW = 512;              // columns per wave
constexpr int ROWB = QKW * 2;         // bytes of one slice row (1 KiB)
constexpr int NKS = QKW / 32;         // k-steps of phase 1 (16)
constexpr int NCT = QKW / 32;         // 32-column tiles of phase 2 (16)
constexpr int PH = 32;                // iterates per workgroup (one half)
constexpr int SLICE = PRB * ROWB;     // 16 KiB
constexpr int XS = PH * 2 + 16;       // X staging row stride (bytes)
constexpr int PF = 4;                 // G tree fan-in
#ifndef MPA_LSQP4_AD
#define MPA_LSQP4_AD 3                // phase-1 fragment read-ahead in k-steps (3 beats 2, 4, 6)
#endif
static_assert(QW * QKW == kLsqpMaxCols, "4 waves x 512 columns");
static_assert(NKS == 16 && NCT == 16, "8 strips of 64 columns per wave");

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// G's 16 tiles are not compiler variables: tile ct is a[16 ct .. 16 ct + 15], named in the
// asm text and declared clobbered by the MFMAs that accumulate into it, so the compiler keeps
// nothing of its own there across them and never moves G.  (As compiler values -- the
// intrinsic, an "a" or a named-tuple constraint -- the allocator spilled ~180 registers around
// the block loop, or moved a tile through VGPRs around the asm MFMAs with accvgpr copies whose
// hazards it does not pad: 2e-4 errors in the general form.)  Hazards are the kernel's: every
// MFMA opens with the 2 wait states a VALU write -> MFMA operand read needs (the reduce's
// permlane swaps, the compiler's copies into the B tuple); a tile's lo MFMA directly follows its
// hi MFMA (the next MFMA taking the result whole as SrcC: no wait states); the tiles are read
// by VALU only after g_settle's 24 wait states, and written (g_zero) long before the first MFMA.
__device__ __forceinline__ void mfma32(int ct, const bf16x8& a, const bf16x8& b) {
  switch (ct) {
    case 0:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[0:15], %0, %1, a[0:15]" ::"v"(a), "v"(b)
                   : "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15");
      break;
    case 1:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[16:31], %0, %1, a[16:31]" ::"v"(a), "v"(b)
                   : "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31");
      break;
    case 2:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[32:47], %0, %1, a[32:47]" ::"v"(a), "v"(b)
                   : "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47");
      break;
    case 3:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[48:63], %0, %1, a[48:63]" ::"v"(a), "v"(b)
                   : "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63");
      break;
    case 4:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[64:79], %0, %1, a[64:79]" ::"v"(a), "v"(b)
                   : "a64", "a65", "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75", "a76", "a77", "a78", "a79");
      break;
    case 5:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[80:95], %0, %1, a[80:95]" ::"v"(a), "v"(b)
                   : "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90", "a91", "a92", "a93", "a94", "a95");
      break;
    case 6:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[96:111], %0, %1, a[96:111]" ::"v"(a), "v"(b)
                   : "a96", "a97", "a98", "a99", "a100", "a101", "a102", "a103", "a104", "a105", "a106", "a107", "a108", "a109", "a110", "a111");
      break;
    case 7:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[112:127], %0, %1, a[112:127]" ::"v"(a), "v"(b)
                   : "a112", "a113", "a114", "a115", "a116", "a117", "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", "a126", "a127");
      break;
    case 8:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[128:143], %0, %1, a[128:143]" ::"v"(a), "v"(b)
                   : "a128", "a129", "a130", "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", "a139", "a140", "a141", "a142", "a143");
      break;
    case 9:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[144:159], %0, %1, a[144:159]" ::"v"(a), "v"(b)
                   : "a144", "a145", "a146", "a147", "a148", "a149", "a150", "a151", "a152", "a153", "a154", "a155", "a156", "a157", "a158", "a159");
      break;
    case 10:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[160:175], %0, %1, a[160:175]" ::"v"(a), "v"(b)
                   : "a160", "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", "a170", "a171", "a172", "a173", "a174", "a175");
      break;
    case 11:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[176:191], %0, %1, a[176:191]" ::"v"(a), "v"(b)
                   : "a176", "a177", "a178", "a179", "a180", "a181", "a182", "a183", "a184", "a185", "a186", "a187", "a188", "a189", "a190", "a191");
      break;
    case 12:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[192:207], %0, %1, a[192:207]" ::"v"(a), "v"(b)
                   : "a192", "a193", "a194", "a195", "a196", "a197", "a198", "a199", "a200", "a201", "a202", "a203", "a204", "a205", "a206", "a207");
      break;
    case 13:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[208:223], %0, %1, a[208:223]" ::"v"(a), "v"(b)
                   : "a208", "a209", "a210", "a211", "a212", "a213", "a214", "a215", "a216", "a217", "a218", "a219", "a220", "a221", "a222", "a223");
      break;
    case 14:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[224:239], %0, %1, a[224:239]" ::"v"(a), "v"(b)
                   : "a224", "a225", "a226", "a227", "a228", "a229", "a230", "a231", "a232", "a233", "a234", "a235", "a236", "a237", "a238", "a239");
      break;
    case 15:
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[240:255], %0, %1, a[240:255]" ::"v"(a), "v"(b)
                   : "a240", "a241", "a242", "a243", "a244", "a245", "a246", "a247", "a248", "a249", "a250", "a251", "a252", "a253", "a254", "a255");
      break;
  }
}
// tile ct into VGPRs (the output stage)
__device__ __forceinline__ f32x16 g_tile(int ct) {
  float x[16];
  switch (ct) {
    case 0:
      asm volatile("v_accvgpr_read_b32 %0, a0\n\tv_accvgpr_read_b32 %1, a1\n\tv_accvgpr_read_b32 %2, a2\n\tv_accvgpr_read_b32 %3, a3\n\tv_accvgpr_read_b32 %4, a4\n\tv_accvgpr_read_b32 %5, a5\n\tv_accvgpr_read_b32 %6, a6\n\tv_accvgpr_read_b32 %7, a7\n\tv_accvgpr_read_b32 %8, a8\n\tv_accvgpr_read_b32 %9, a9\n\tv_accvgpr_read_b32 %10, a10\n\tv_accvgpr_read_b32 %11, a11\n\tv_accvgpr_read_b32 %12, a12\n\tv_accvgpr_read_b32 %13, a13\n\tv_accvgpr_read_b32 %14, a14\n\tv_accvgpr_read_b32 %15, a15"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 1:
      asm volatile("v_accvgpr_read_b32 %0, a16\n\tv_accvgpr_read_b32 %1, a17\n\tv_accvgpr_read_b32 %2, a18\n\tv_accvgpr_read_b32 %3, a19\n\tv_accvgpr_read_b32 %4, a20\n\tv_accvgpr_read_b32 %5, a21\n\tv_accvgpr_read_b32 %6, a22\n\tv_accvgpr_read_b32 %7, a23\n\tv_accvgpr_read_b32 %8, a24\n\tv_accvgpr_read_b32 %9, a25\n\tv_accvgpr_read_b32 %10, a26\n\tv_accvgpr_read_b32 %11, a27\n\tv_accvgpr_read_b32 %12, a28\n\tv_accvgpr_read_b32 %13, a29\n\tv_accvgpr_read_b32 %14, a30\n\tv_accvgpr_read_b32 %15, a31"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 2:
      asm volatile("v_accvgpr_read_b32 %0, a32\n\tv_accvgpr_read_b32 %1, a33\n\tv_accvgpr_read_b32 %2, a34\n\tv_accvgpr_read_b32 %3, a35\n\tv_accvgpr_read_b32 %4, a36\n\tv_accvgpr_read_b32 %5, a37\n\tv_accvgpr_read_b32 %6, a38\n\tv_accvgpr_read_b32 %7, a39\n\tv_accvgpr_read_b32 %8, a40\n\tv_accvgpr_read_b32 %9, a41\n\tv_accvgpr_read_b32 %10, a42\n\tv_accvgpr_read_b32 %11, a43\n\tv_accvgpr_read_b32 %12, a44\n\tv_accvgpr_read_b32 %13, a45\n\tv_accvgpr_read_b32 %14, a46\n\tv_accvgpr_read_b32 %15, a47"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 3:
      asm volatile("v_accvgpr_read_b32 %0, a48\n\tv_accvgpr_read_b32 %1, a49\n\tv_accvgpr_read_b32 %2, a50\n\tv_accvgpr_read_b32 %3, a51\n\tv_accvgpr_read_b32 %4, a52\n\tv_accvgpr_read_b32 %5, a53\n\tv_accvgpr_read_b32 %6, a54\n\tv_accvgpr_read_b32 %7, a55\n\tv_accvgpr_read_b32 %8, a56\n\tv_accvgpr_read_b32 %9, a57\n\tv_accvgpr_read_b32 %10, a58\n\tv_accvgpr_read_b32 %11, a59\n\tv_accvgpr_read_b32 %12, a60\n\tv_accvgpr_read_b32 %13, a61\n\tv_accvgpr_read_b32 %14, a62\n\tv_accvgpr_read_b32 %15, a63"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 4:
      asm volatile("v_accvgpr_read_b32 %0, a64\n\tv_accvgpr_read_b32 %1, a65\n\tv_accvgpr_read_b32 %2, a66\n\tv_accvgpr_read_b32 %3, a67\n\tv_accvgpr_read_b32 %4, a68\n\tv_accvgpr_read_b32 %5, a69\n\tv_accvgpr_read_b32 %6, a70\n\tv_accvgpr_read_b32 %7, a71\n\tv_accvgpr_read_b32 %8, a72\n\tv_accvgpr_read_b32 %9, a73\n\tv_accvgpr_read_b32 %10, a74\n\tv_accvgpr_read_b32 %11, a75\n\tv_accvgpr_read_b32 %12, a76\n\tv_accvgpr_read_b32 %13, a77\n\tv_accvgpr_read_b32 %14, a78\n\tv_accvgpr_read_b32 %15, a79"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 5:
      asm volatile("v_accvgpr_read_b32 %0, a80\n\tv_accvgpr_read_b32 %1, a81\n\tv_accvgpr_read_b32 %2, a82\n\tv_accvgpr_read_b32 %3, a83\n\tv_accvgpr_read_b32 %4, a84\n\tv_accvgpr_read_b32 %5, a85\n\tv_accvgpr_read_b32 %6, a86\n\tv_accvgpr_read_b32 %7, a87\n\tv_accvgpr_read_b32 %8, a88\n\tv_accvgpr_read_b32 %9, a89\n\tv_accvgpr_read_b32 %10, a90\n\tv_accvgpr_read_b32 %11, a91\n\tv_accvgpr_read_b32 %12, a92\n\tv_accvgpr_read_b32 %13, a93\n\tv_accvgpr_read_b32 %14, a94\n\tv_accvgpr_read_b32 %15, a95"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 6:
      asm volatile("v_accvgpr_read_b32 %0, a96\n\tv_accvgpr_read_b32 %1, a97\n\tv_accvgpr_read_b32 %2, a98\n\tv_accvgpr_read_b32 %3, a99\n\tv_accvgpr_read_b32 %4, a100\n\tv_accvgpr_read_b32 %5, a101\n\tv_accvgpr_read_b32 %6, a102\n\tv_accvgpr_read_b32 %7, a103\n\tv_accvgpr_read_b32 %8, a104\n\tv_accvgpr_read_b32 %9, a105\n\tv_accvgpr_read_b32 %10, a106\n\tv_accvgpr_read_b32 %11, a107\n\tv_accvgpr_read_b32 %12, a108\n\tv_accvgpr_read_b32 %13, a109\n\tv_accvgpr_read_b32 %14, a110\n\tv_accvgpr_read_b32 %15, a111"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 7:
      asm volatile("v_accvgpr_read_b32 %0, a112\n\tv_accvgpr_read_b32 %1, a113\n\tv_accvgpr_read_b32 %2, a114\n\tv_accvgpr_read_b32 %3, a115\n\tv_accvgpr_read_b32 %4, a116\n\tv_accvgpr_read_b32 %5, a117\n\tv_accvgpr_read_b32 %6, a118\n\tv_accvgpr_read_b32 %7, a119\n\tv_accvgpr_read_b32 %8, a120\n\tv_accvgpr_read_b32 %9, a121\n\tv_accvgpr_read_b32 %10, a122\n\tv_accvgpr_read_b32 %11, a123\n\tv_accvgpr_read_b32 %12, a124\n\tv_accvgpr_read_b32 %13, a125\n\tv_accvgpr_read_b32 %14, a126\n\tv_accvgpr_read_b32 %15, a127"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 8:
      asm volatile("v_accvgpr_read_b32 %0, a128\n\tv_accvgpr_read_b32 %1, a129\n\tv_accvgpr_read_b32 %2, a130\n\tv_accvgpr_read_b32 %3, a131\n\tv_accvgpr_read_b32 %4, a132\n\tv_accvgpr_read_b32 %5, a133\n\tv_accvgpr_read_b32 %6, a134\n\tv_accvgpr_read_b32 %7, a135\n\tv_accvgpr_read_b32 %8, a136\n\tv_accvgpr_read_b32 %9, a137\n\tv_accvgpr_read_b32 %10, a138\n\tv_accvgpr_read_b32 %11, a139\n\tv_accvgpr_read_b32 %12, a140\n\tv_accvgpr_read_b32 %13, a141\n\tv_accvgpr_read_b32 %14, a142\n\tv_accvgpr_read_b32 %15, a143"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 9:
      asm volatile("v_accvgpr_read_b32 %0, a144\n\tv_accvgpr_read_b32 %1, a145\n\tv_accvgpr_read_b32 %2, a146\n\tv_accvgpr_read_b32 %3, a147\n\tv_accvgpr_read_b32 %4, a148\n\tv_accvgpr_read_b32 %5, a149\n\tv_accvgpr_read_b32 %6, a150\n\tv_accvgpr_read_b32 %7, a151\n\tv_accvgpr_read_b32 %8, a152\n\tv_accvgpr_read_b32 %9, a153\n\tv_accvgpr_read_b32 %10, a154\n\tv_accvgpr_read_b32 %11, a155\n\tv_accvgpr_read_b32 %12, a156\n\tv_accvgpr_read_b32 %13, a157\n\tv_accvgpr_read_b32 %14, a158\n\tv_accvgpr_read_b32 %15, a159"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 10:
      asm volatile("v_accvgpr_read_b32 %0, a160\n\tv_accvgpr_read_b32 %1, a161\n\tv_accvgpr_read_b32 %2, a162\n\tv_accvgpr_read_b32 %3, a163\n\tv_accvgpr_read_b32 %4, a164\n\tv_accvgpr_read_b32 %5, a165\n\tv_accvgpr_read_b32 %6, a166\n\tv_accvgpr_read_b32 %7, a167\n\tv_accvgpr_read_b32 %8, a168\n\tv_accvgpr_read_b32 %9, a169\n\tv_accvgpr_read_b32 %10, a170\n\tv_accvgpr_read_b32 %11, a171\n\tv_accvgpr_read_b32 %12, a172\n\tv_accvgpr_read_b32 %13, a173\n\tv_accvgpr_read_b32 %14, a174\n\tv_accvgpr_read_b32 %15, a175"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 11:
      asm volatile("v_accvgpr_read_b32 %0, a176\n\tv_accvgpr_read_b32 %1, a177\n\tv_accvgpr_read_b32 %2, a178\n\tv_accvgpr_read_b32 %3, a179\n\tv_accvgpr_read_b32 %4, a180\n\tv_accvgpr_read_b32 %5, a181\n\tv_accvgpr_read_b32 %6, a182\n\tv_accvgpr_read_b32 %7, a183\n\tv_accvgpr_read_b32 %8, a184\n\tv_accvgpr_read_b32 %9, a185\n\tv_accvgpr_read_b32 %10, a186\n\tv_accvgpr_read_b32 %11, a187\n\tv_accvgpr_read_b32 %12, a188\n\tv_accvgpr_read_b32 %13, a189\n\tv_accvgpr_read_b32 %14, a190\n\tv_accvgpr_read_b32 %15, a191"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 12:
      asm volatile("v_accvgpr_read_b32 %0, a192\n\tv_accvgpr_read_b32 %1, a193\n\tv_accvgpr_read_b32 %2, a194\n\tv_accvgpr_read_b32 %3, a195\n\tv_accvgpr_read_b32 %4, a196\n\tv_accvgpr_read_b32 %5, a197\n\tv_accvgpr_read_b32 %6, a198\n\tv_accvgpr_read_b32 %7, a199\n\tv_accvgpr_read_b32 %8, a200\n\tv_accvgpr_read_b32 %9, a201\n\tv_accvgpr_read_b32 %10, a202\n\tv_accvgpr_read_b32 %11, a203\n\tv_accvgpr_read_b32 %12, a204\n\tv_accvgpr_read_b32 %13, a205\n\tv_accvgpr_read_b32 %14, a206\n\tv_accvgpr_read_b32 %15, a207"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 13:
      asm volatile("v_accvgpr_read_b32 %0, a208\n\tv_accvgpr_read_b32 %1, a209\n\tv_accvgpr_read_b32 %2, a210\n\tv_accvgpr_read_b32 %3, a211\n\tv_accvgpr_read_b32 %4, a212\n\tv_accvgpr_read_b32 %5, a213\n\tv_accvgpr_read_b32 %6, a214\n\tv_accvgpr_read_b32 %7, a215\n\tv_accvgpr_read_b32 %8, a216\n\tv_accvgpr_read_b32 %9, a217\n\tv_accvgpr_read_b32 %10, a218\n\tv_accvgpr_read_b32 %11, a219\n\tv_accvgpr_read_b32 %12, a220\n\tv_accvgpr_read_b32 %13, a221\n\tv_accvgpr_read_b32 %14, a222\n\tv_accvgpr_read_b32 %15, a223"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 14:
      asm volatile("v_accvgpr_read_b32 %0, a224\n\tv_accvgpr_read_b32 %1, a225\n\tv_accvgpr_read_b32 %2, a226\n\tv_accvgpr_read_b32 %3, a227\n\tv_accvgpr_read_b32 %4, a228\n\tv_accvgpr_read_b32 %5, a229\n\tv_accvgpr_read_b32 %6, a230\n\tv_accvgpr_read_b32 %7, a231\n\tv_accvgpr_read_b32 %8, a232\n\tv_accvgpr_read_b32 %9, a233\n\tv_accvgpr_read_b32 %10, a234\n\tv_accvgpr_read_b32 %11, a235\n\tv_accvgpr_read_b32 %12, a236\n\tv_accvgpr_read_b32 %13, a237\n\tv_accvgpr_read_b32 %14, a238\n\tv_accvgpr_read_b32 %15, a239"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
    case 15:
      asm volatile("v_accvgpr_read_b32 %0, a240\n\tv_accvgpr_read_b32 %1, a241\n\tv_accvgpr_read_b32 %2, a242\n\tv_accvgpr_read_b32 %3, a243\n\tv_accvgpr_read_b32 %4, a244\n\tv_accvgpr_read_b32 %5, a245\n\tv_accvgpr_read_b32 %6, a246\n\tv_accvgpr_read_b32 %7, a247\n\tv_accvgpr_read_b32 %8, a248\n\tv_accvgpr_read_b32 %9, a249\n\tv_accvgpr_read_b32 %10, a250\n\tv_accvgpr_read_b32 %11, a251\n\tv_accvgpr_read_b32 %12, a252\n\tv_accvgpr_read_b32 %13, a253\n\tv_accvgpr_read_b32 %14, a254\n\tv_accvgpr_read_b32 %15, a255"
                   : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7]), "=v"(x[8]), "=v"(x[9]), "=v"(x[10]), "=v"(x[11]), "=v"(x[12]), "=v"(x[13]), "=v"(x[14]), "=v"(x[15]));
      break;
  }
  f32x16 v;
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = x[j];
  return v;
}
__device__ __forceinline__ void g_zero() {
  asm volatile("v_accvgpr_write_b32 a0, 0\n\tv_accvgpr_write_b32 a1, 0\n\tv_accvgpr_write_b32 a2, 0\n\tv_accvgpr_write_b32 a3, 0\n\tv_accvgpr_write_b32 a4, 0\n\tv_accvgpr_write_b32 a5, 0\n\tv_accvgpr_write_b32 a6, 0\n\tv_accvgpr_write_b32 a7, 0\n\tv_accvgpr_write_b32 a8, 0\n\tv_accvgpr_write_b32 a9, 0\n\tv_accvgpr_write_b32 a10, 0\n\tv_accvgpr_write_b32 a11, 0\n\tv_accvgpr_write_b32 a12, 0\n\tv_accvgpr_write_b32 a13, 0\n\tv_accvgpr_write_b32 a14, 0\n\tv_accvgpr_write_b32 a15, 0\n\tv_accvgpr_write_b32 a16, 0\n\tv_accvgpr_write_b32 a17, 0\n\tv_accvgpr_write_b32 a18, 0\n\tv_accvgpr_write_b32 a19, 0\n\tv_accvgpr_write_b32 a20, 0\n\tv_accvgpr_write_b32 a21, 0\n\tv_accvgpr_write_b32 a22, 0\n\tv_accvgpr_write_b32 a23, 0\n\tv_accvgpr_write_b32 a24, 0\n\tv_accvgpr_write_b32 a25, 0\n\tv_accvgpr_write_b32 a26, 0\n\tv_accvgpr_write_b32 a27, 0\n\tv_accvgpr_write_b32 a28, 0\n\tv_accvgpr_write_b32 a29, 0\n\tv_accvgpr_write_b32 a30, 0\n\tv_accvgpr_write_b32 a31, 0\n\tv_accvgpr_write_b32 a32, 0\n\tv_accvgpr_write_b32 a33, 0\n\tv_accvgpr_write_b32 a34, 0\n\tv_accvgpr_write_b32 a35, 0\n\tv_accvgpr_write_b32 a36, 0\n\tv_accvgpr_write_b32 a37, 0\n\tv_accvgpr_write_b32 a38, 0\n\tv_accvgpr_write_b32 a39, 0\n\tv_accvgpr_write_b32 a40, 0\n\tv_accvgpr_write_b32 a41, 0\n\tv_accvgpr_write_b32 a42, 0\n\tv_accvgpr_write_b32 a43, 0\n\tv_accvgpr_write_b32 a44, 0\n\tv_accvgpr_write_b32 a45, 0\n\tv_accvgpr_write_b32 a46, 0\n\tv_accvgpr_write_b32 a47, 0\n\tv_accvgpr_write_b32 a48, 0\n\tv_accvgpr_write_b32 a49, 0\n\tv_accvgpr_write_b32 a50, 0\n\tv_accvgpr_write_b32 a51, 0\n\tv_accvgpr_write_b32 a52, 0\n\tv_accvgpr_write_b32 a53, 0\n\tv_accvgpr_write_b32 a54, 0\n\tv_accvgpr_write_b32 a55, 0\n\tv_accvgpr_write_b32 a56, 0\n\tv_accvgpr_write_b32 a57, 0\n\tv_accvgpr_write_b32 a58, 0\n\tv_accvgpr_write_b32 a59, 0\n\tv_accvgpr_write_b32 a60, 0\n\tv_accvgpr_write_b32 a61, 0\n\tv_accvgpr_write_b32 a62, 0\n\tv_accvgpr_write_b32 a63, 0\n\tv_accvgpr_write_b32 a64, 0\n\tv_accvgpr_write_b32 a65, 0\n\tv_accvgpr_write_b32 a66, 0\n\tv_accvgpr_write_b32 a67, 0\n\tv_accvgpr_write_b32 a68, 0\n\tv_accvgpr_write_b32 a69, 0\n\tv_accvgpr_write_b32 a70, 0\n\tv_accvgpr_write_b32 a71, 0\n\tv_accvgpr_write_b32 a72, 0\n\tv_accvgpr_write_b32 a73, 0\n\tv_accvgpr_write_b32 a74, 0\n\tv_accvgpr_write_b32 a75, 0\n\tv_accvgpr_write_b32 a76, 0\n\tv_accvgpr_write_b32 a77, 0\n\tv_accvgpr_write_b32 a78, 0\n\tv_accvgpr_write_b32 a79, 0\n\tv_accvgpr_write_b32 a80, 0\n\tv_accvgpr_write_b32 a81, 0\n\tv_accvgpr_write_b32 a82, 0\n\tv_accvgpr_write_b32 a83, 0\n\tv_accvgpr_write_b32 a84, 0\n\tv_accvgpr_write_b32 a85, 0\n\tv_accvgpr_write_b32 a86, 0\n\tv_accvgpr_write_b32 a87, 0\n\tv_accvgpr_write_b32 a88, 0\n\tv_accvgpr_write_b32 a89, 0\n\tv_accvgpr_write_b32 a90, 0\n\tv_accvgpr_write_b32 a91, 0\n\tv_accvgpr_write_b32 a92, 0\n\tv_accvgpr_write_b32 a93, 0\n\tv_accvgpr_write_b32 a94, 0\n\tv_accvgpr_write_b32 a95, 0\n\tv_accvgpr_write_b32 a96, 0\n\tv_accvgpr_write_b32 a97, 0\n\tv_accvgpr_write_b32 a98, 0\n\tv_accvgpr_write_b32 a99, 0\n\tv_accvgpr_write_b32 a100, 0\n\tv_accvgpr_write_b32 a101, 0\n\tv_accvgpr_write_b32 a102, 0\n\tv_accvgpr_write_b32 a103, 0\n\tv_accvgpr_write_b32 a104, 0\n\tv_accvgpr_write_b32 a105, 0\n\tv_accvgpr_write_b32 a106, 0\n\tv_accvgpr_write_b32 a107, 0\n\tv_accvgpr_write_b32 a108, 0\n\tv_accvgpr_write_b32 a109, 0\n\tv_accvgpr_write_b32 a110, 0\n\tv_accvgpr_write_b32 a111, 0\n\tv_accvgpr_write_b32 a112, 0\n\tv_accvgpr_write_b32 a113, 0\n\tv_accvgpr_write_b32 a114, 0\n\tv_accvgpr_write_b32 a115, 0\n\tv_accvgpr_write_b32 a116, 0\n\tv_accvgpr_write_b32 a117, 0\n\tv_accvgpr_write_b32 a118, 0\n\tv_accvgpr_write_b32 a119, 0\n\tv_accvgpr_write_b32 a120, 0\n\tv_accvgpr_write_b32 a121, 0\n\tv_accvgpr_write_b32 a122, 0\n\tv_accvgpr_write_b32 a123, 0\n\tv_accvgpr_write_b32 a124, 0\n\tv_accvgpr_write_b32 a125, 0\n\tv_accvgpr_write_b32 a126, 0\n\tv_accvgpr_write_b32 a127, 0\n\tv_accvgpr_write_b32 a128, 0\n\tv_accvgpr_write_b32 a129, 0\n\tv_accvgpr_write_b32 a130, 0\n\tv_accvgpr_write_b32 a131, 0\n\tv_accvgpr_write_b32 a132, 0\n\tv_accvgpr_write_b32 a133, 0\n\tv_accvgpr_write_b32 a134, 0\n\tv_accvgpr_write_b32 a135, 0\n\tv_accvgpr_write_b32 a136, 0\n\tv_accvgpr_write_b32 a137, 0\n\tv_accvgpr_write_b32 a138, 0\n\tv_accvgpr_write_b32 a139, 0\n\tv_accvgpr_write_b32 a140, 0\n\tv_accvgpr_write_b32 a141, 0\n\tv_accvgpr_write_b32 a142, 0\n\tv_accvgpr_write_b32 a143, 0\n\tv_accvgpr_write_b32 a144, 0\n\tv_accvgpr_write_b32 a145, 0\n\tv_accvgpr_write_b32 a146, 0\n\tv_accvgpr_write_b32 a147, 0\n\tv_accvgpr_write_b32 a148, 0\n\tv_accvgpr_write_b32 a149, 0\n\tv_accvgpr_write_b32 a150, 0\n\tv_accvgpr_write_b32 a151, 0\n\tv_accvgpr_write_b32 a152, 0\n\tv_accvgpr_write_b32 a153, 0\n\tv_accvgpr_write_b32 a154, 0\n\tv_accvgpr_write_b32 a155, 0\n\tv_accvgpr_write_b32 a156, 0\n\tv_accvgpr_write_b32 a157, 0\n\tv_accvgpr_write_b32 a158, 0\n\tv_accvgpr_write_b32 a159, 0\n\tv_accvgpr_write_b32 a160, 0\n\tv_accvgpr_write_b32 a161, 0\n\tv_accvgpr_write_b32 a162, 0\n\tv_accvgpr_write_b32 a163, 0\n\tv_accvgpr_write_b32 a164, 0\n\tv_accvgpr_write_b32 a165, 0\n\tv_accvgpr_write_b32 a166, 0\n\tv_accvgpr_write_b32 a167, 0\n\tv_accvgpr_write_b32 a168, 0\n\tv_accvgpr_write_b32 a169, 0\n\tv_accvgpr_write_b32 a170, 0\n\tv_accvgpr_write_b32 a171, 0\n\tv_accvgpr_write_b32 a172, 0\n\tv_accvgpr_write_b32 a173, 0\n\tv_accvgpr_write_b32 a174, 0\n\tv_accvgpr_write_b32 a175, 0\n\tv_accvgpr_write_b32 a176, 0\n\tv_accvgpr_write_b32 a177, 0\n\tv_accvgpr_write_b32 a178, 0\n\tv_accvgpr_write_b32 a179, 0\n\tv_accvgpr_write_b32 a180, 0\n\tv_accvgpr_write_b32 a181, 0\n\tv_accvgpr_write_b32 a182, 0\n\tv_accvgpr_write_b32 a183, 0\n\tv_accvgpr_write_b32 a184, 0\n\tv_accvgpr_write_b32 a185, 0\n\tv_accvgpr_write_b32 a186, 0\n\tv_accvgpr_write_b32 a187, 0\n\tv_accvgpr_write_b32 a188, 0\n\tv_accvgpr_write_b32 a189, 0\n\tv_accvgpr_write_b32 a190, 0\n\tv_accvgpr_write_b32 a191, 0\n\tv_accvgpr_write_b32 a192, 0\n\tv_accvgpr_write_b32 a193, 0\n\tv_accvgpr_write_b32 a194, 0\n\tv_accvgpr_write_b32 a195, 0\n\tv_accvgpr_write_b32 a196, 0\n\tv_accvgpr_write_b32 a197, 0\n\tv_accvgpr_write_b32 a198, 0\n\tv_accvgpr_write_b32 a199, 0\n\tv_accvgpr_write_b32 a200, 0\n\tv_accvgpr_write_b32 a201, 0\n\tv_accvgpr_write_b32 a202, 0\n\tv_accvgpr_write_b32 a203, 0\n\tv_accvgpr_write_b32 a204, 0\n\tv_accvgpr_write_b32 a205, 0\n\tv_accvgpr_write_b32 a206, 0\n\tv_accvgpr_write_b32 a207, 0\n\tv_accvgpr_write_b32 a208, 0\n\tv_accvgpr_write_b32 a209, 0\n\tv_accvgpr_write_b32 a210, 0\n\tv_accvgpr_write_b32 a211, 0\n\tv_accvgpr_write_b32 a212, 0\n\tv_accvgpr_write_b32 a213, 0\n\tv_accvgpr_write_b32 a214, 0\n\tv_accvgpr_write_b32 a215, 0\n\tv_accvgpr_write_b32 a216, 0\n\tv_accvgpr_write_b32 a217, 0\n\tv_accvgpr_write_b32 a218, 0\n\tv_accvgpr_write_b32 a219, 0\n\tv_accvgpr_write_b32 a220, 0\n\tv_accvgpr_write_b32 a221, 0\n\tv_accvgpr_write_b32 a222, 0\n\tv_accvgpr_write_b32 a223, 0\n\tv_accvgpr_write_b32 a224, 0\n\tv_accvgpr_write_b32 a225, 0\n\tv_accvgpr_write_b32 a226, 0\n\tv_accvgpr_write_b32 a227, 0\n\tv_accvgpr_write_b32 a228, 0\n\tv_accvgpr_write_b32 a229, 0\n\tv_accvgpr_write_b32 a230, 0\n\tv_accvgpr_write_b32 a231, 0\n\tv_accvgpr_write_b32 a232, 0\n\tv_accvgpr_write_b32 a233, 0\n\tv_accvgpr_write_b32 a234, 0\n\tv_accvgpr_write_b32 a235, 0\n\tv_accvgpr_write_b32 a236, 0\n\tv_accvgpr_write_b32 a237, 0\n\tv_accvgpr_write_b32 a238, 0\n\tv_accvgpr_write_b32 a239, 0\n\tv_accvgpr_write_b32 a240, 0\n\tv_accvgpr_write_b32 a241, 0\n\tv_accvgpr_write_b32 a242, 0\n\tv_accvgpr_write_b32 a243, 0\n\tv_accvgpr_write_b32 a244, 0\n\tv_accvgpr_write_b32 a245, 0\n\tv_accvgpr_write_b32 a246, 0\n\tv_accvgpr_write_b32 a247, 0\n\tv_accvgpr_write_b32 a248, 0\n\tv_accvgpr_write_b32 a249, 0\n\tv_accvgpr_write_b32 a250, 0\n\tv_accvgpr_write_b32 a251, 0\n\tv_accvgpr_write_b32 a252, 0\n\tv_accvgpr_write_b32 a253, 0\n\tv_accvgpr_write_b32 a254, 0\n\tv_accvgpr_write_b32 a255, 0\n\ts_nop 7" ::: "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47", "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63", "a64", "a65", "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75", "a76", "a77", "a78", "a79", "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90", "a91", "a92", "a93", "a94", "a95", "a96", "a97", "a98", "a99", "a100", "a101", "a102", "a103", "a104", "a105", "a106", "a107", "a108", "a109", "a110", "a111", "a112", "a113", "a114", "a115", "a116", "a117", "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", "a126", "a127", "a128", "a129", "a130", "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", "a139", "a140", "a141", "a142", "a143", "a144", "a145", "a146", "a147", "a148", "a149", "a150", "a151", "a152", "a153", "a154", "a155", "a156", "a157", "a158", "a159", "a160", "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", "a170", "a171", "a172", "a173", "a174", "a175", "a176", "a177", "a178", "a179", "a180", "a181", "a182", "a183", "a184", "a185", "a186", "a187", "a188", "a189", "a190", "a191", "a192", "a193", "a194", "a195", "a196", "a197", "a198", "a199", "a200", "a201", "a202", "a203", "a204", "a205", "a206", "a207", "a208", "a209", "a210", "a211", "a212", "a213", "a214", "a215", "a216", "a217", "a218", "a219", "a220", "a221", "a222", "a223", "a224", "a225", "a226", "a227", "a228", "a229", "a230", "a231", "a232", "a233", "a234", "a235", "a236", "a237", "a238", "a239", "a240", "a241", "a242", "a243", "a244", "a245", "a246", "a247", "a248", "a249", "a250", "a251", "a252", "a253", "a254", "a255");
}
__device__ __forceinline__ void g_settle() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }
// MPA_LSQP4_PROBE (timing-probe builds only, wrong results: make BUILD=... EXTRA=-DMPA_LSQP4_PROBE=n,
// profiles/r03_c5_probes.txt): 1 no strip DMAs in the block loop, 2 no cross-wave exchange /
// barrier in the reduce, 4 no phase-1 MFMAs
#ifndef MPA_LSQP4_PROBE
#define MPA_LSQP4_PROBE 0
#endif
#ifndef MPA_LSQP4_VACC
#define MPA_LSQP4_VACC 1  // phase-1 accumulators in VGPRs (inline asm MFMAs)
#endif
// Phase 1's accumulators in VGPRs.  G takes all 256 AGPRs, and the compiler gives every MFMA
// intrinsic AGPR accumulators, so with intrinsics it parks 8 G registers in VGPRs around every
// phase 1 (24 moves per block).  These asm forms keep the phase-1 chain in VGPRs.  Hazards are
// the kernel's (the compiler does not look inside): the chain reads its own previous result as
// SrcC (exact overlap: back to back is allowed), A / B operands come from LDS reads (lgkmcnt,
// which the compiler does insert for asm operands) or registers written long before; the one
// non-MFMA reader of the result gets 16 wait states first (mfma_v_settle)
__device__ __forceinline__ f32x4 mfma_v0(const bf16x8& a, const bf16x8& b) {
  f32x4 d;
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ void mfma_v(f32x4& d, const bf16x8& a, const bf16x8& b) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_v_settle(f32x4& d0, f32x4& d1) {
  asm volatile("s_nop 7\n\ts_nop 7" : "+v"(d0), "+v"(d1));
}
__device__ __forceinline__ void lgkm_drain() { __builtin_amdgcn_s_waitcnt(0xc07f); }  // lgkmcnt(0)
// lgkmcnt(N) alone (vmcnt / expcnt fields left free)
template <int N>
__device__ __forceinline__ void lgkm_wait() {
  static_assert(N >= 0 && N < 16, "lgkmcnt is 4 bits");
  __builtin_amdgcn_s_waitcnt(0xc07f | (N << 8));
}
// workgroup barrier that leaves the vector-memory queue alone (the next block's DMA stays in
// flight): LDS traffic drained, then s_barrier; the clobber pins LDS accesses on either side
__device__ __forceinline__ void barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA of one 1-KiB slice row: lane l's 16 B land at lds + 16 l.  Scalar base + 32-bit lane
// offset (the saddr form).  Inline asm on purpose, as in lsqp_kernel.hip: the compiler would
// guard every LDS read that may alias a DMA it knows of with vmcnt(0), waiting for the NEXT
// block too; the kernel orders its reads itself (vmcnt per block).
__device__ __forceinline__ void dma_row(const void* sbase, uint32_t voff, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(l) : "memory");
}
__device__ __forceinline__ void pf4(const void* src, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(l) : "memory");
}
__device__ __forceinline__ void dma16(const void* src, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(l) : "memory");
}
// the saddr forms with an immediate offset (FULL blocks): the instruction adds OFF to the
// global address AND to the LDS address (llvm.amdgcn.global.load.lds: "applied to both"), so
// m0 = LDS destination - OFF.  One scalar base per block instead of a 64-bit add per strip
// A whole strip (both halves) under one M0 write: half j lands at lds + 1024 j and reads its
// rows at voff_j, so with m0 = lds - OFF and offsets OFF and OFF + 1024 the second half's lane
// offset is passed as voff_1 - 1024 (voff_1 >= 8 rows >= 1024 B)
template <int OFF>
__device__ __forceinline__ void dma_strip_off(const void* sbase, uint32_t voff0, uint32_t voff1m, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds))) - uint32_t(OFF);
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %2 offset:%4\n\t"
               "global_load_lds_dwordx4 %1, %2 offset:%5"
               ::"v"(voff0), "v"(voff1m), "s"(sbase), "s"(l), "i"(OFF), "i"(OFF + 1024) : "memory");
}
__device__ __forceinline__ void dma16_s(const void* sbase, uint32_t voff, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(l) : "memory");
}
__device__ __forceinline__ void pf4_s(const void* sbase, uint32_t voff, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>(lds)));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(voff), "s"(sbase), "s"(l) : "memory");
}

// 16-B chunk c of strip row r sits at chunk position c ^ sw(r); found by search over the linear
// maps of r's bits for conflict-free reads of both phases: phase 1's 16x16x32 row reads and
// phase 2's 32x32x16 transposed reads (tools/lsqp4_swizzle.py --p5).  sw depends on row bits 1
// and 3 only, which the transposed reads of one tile share, so rows +4 are at +512 B
__host__ __device__ constexpr int sw(int r) { return 4 * ((r >> 1) & 1) + 2 * ((r >> 3) & 1); }

// write-through 16-B store / load as two 8-B agent-scope accesses (the G tree's hand-off:
// MI355X_MICROARCH.md §inter-workgroup visibility, "one lane adds for the producer, the last
// adder loads")
__device__ __forceinline__ void st_wt(f32x4* p, const f32x4& v) {
  const unsigned long long* s = reinterpret_cast<const unsigned long long*>(&v);
  unsigned long long* d = reinterpret_cast<unsigned long long*>(p);
  __hip_atomic_store(d, s[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(d + 1, s[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ f32x4 ld_wt(const f32x4* p) {
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
  unsigned long long u[2];
  u[0] = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  u[1] = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_bit_cast(f32x4, u);
}

// FULL: every task of the batch has cols == 2048 and rows % 16 == 0 (BASELINE c5's shape):
// no ragged block, no partial strip, so the block loop drops the clamps, selects and masks
// of the general form and addresses a block from ONE scalar base (immediate strip offsets)
template <bool ARMED, bool FULL>
__global__ void __launch_bounds__(QT, 1) lsqp5_kernel(LsqpBatch batch) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[QW][2][SLICE];
  __shared__ __attribute__((aligned(16))) uint8_t bring[2][PRB * PH * 2];
  // phase-1 partials, double-buffered by block parity: with one barrier per block, a wave
  // may store block u + 1's partial while a slower wave still reads block u's
  __shared__ __attribute__((aligned(16))) f32x4 part[2][QW][2][64];
  __shared__ __attribute__((aligned(16))) uint32_t sink[QW][64];
  // zeros in B's slot layout, one per wave (each wave zeroes its own: no barrier): the -B MFMA
  // operand of waves 1-3 (MPA_LSQP4_VACC)
  __shared__ __attribute__((aligned(16))) uint8_t bzero[QW][PRB * PH * 2];

  // blocks b and b + 8 are the two halves of one pair (one XCD under round-robin placement;
  // speed only): pair index = (b / 16) * 8 + b % 8
  const int bx = int(blockIdx.x);
  const int h = (bx >> 3) & 1;
  const int pidx = (bx >> 4) * 8 + (bx & 7);
  if (pidx >= batch.grp0[batch.ntasks]) return;  // grid padding (whole workgroup)
  int ti = 0;
  while (ti + 1 < batch.ntasks && pidx >= batch.grp0[ti + 1]) ++ti;
  const LsqpTask& a = batch.t[ti];
  // a pre-armed task its server cancelled computes but neither writes G nor publishes: the
  // go word (host memory) is read once per writing wave at the end (disarmed() below), not by
  // every workgroup before any work (profiles/r02_arm_go_word.txt)
  const int q = pidx - batch.grp0[ti];
  const int ng = batch.grp0[ti + 1] - batch.grp0[ti];
  if constexpr (ARMED)
    if (!wait_door(a.door, a.seq, batch.spin_ticks, batch.err)) return;  // device-armed

  const int tid = threadIdx.x, lane = tid & 63, i = lane & 15, g = lane >> 4;
  const int qq = (lane >> 2) & 3, p4 = lane & 3;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t rows = a.rows;
  const int cols = a.cols;
  const int c0 = w * QKW;
  // valid k-steps of this wave; the loops always run all of them (k-steps past cols meet
  // X = 0, their G columns are never stored): branch-free block loop
  const int nks = cols > c0 ? ((cols - c0) < QKW ? (cols - c0) : QKW) / 32 : 0;
  const int64_t nblocks = (rows + PRB - 1) / PRB;
  // wave-uniform by construction; readfirstlane keeps the block arithmetic on the scalar unit
  // block indices in 32 bits (SALU has no 64-bit compare): the clamps below stay scalar
  const int kb0 = __builtin_amdgcn_readfirstlane(int(nblocks * q / ng)),
            kb1 = __builtin_amdgcn_readfirstlane(int(nblocks * (q + 1) / ng));
  const int kblast = kb1 > kb0 ? kb1 - 1 : kb0;  // past the range, DMAs re-read this block
  const int nb = int(kb1 - kb0);
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(a.A);
  const uint16_t* __restrict__ Bm = static_cast<const uint16_t*>(a.B);
  const uint8_t* __restrict__ X = static_cast<const uint8_t*>(a.X);
  uint8_t* my0 = &ring[w][0][0];
  uint8_t* my1 = &ring[w][1][0];

  // ---- X_h slice -> XF, through the wave's two ring slots (32 KiB) in two rounds of eight
  // k-steps (32 X rows x 64 B each, row stride XS)
  bf16x8 XF[NKS][2];
#pragma unroll
  for (int rd = 0; rd < 2; ++rd) {
    uint4 xr[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int s = 8 * rd + (e >> 1), piece = lane + 64 * (e & 1), r = piece >> 2, c16 = piece & 3;
      xr[e] = s < nks ? *reinterpret_cast<const uint4*>(X + (size_t(c0 + 32 * s + r) * K + PH * h) * 2 + c16 * 16)
                      : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int piece = lane + 64 * (e & 1), r = piece >> 2, c16 = piece & 3;
      *reinterpret_cast<uint4*>(my0 + ((e >> 1) * 32 + r) * XS + c16 * 16) = xr[e];
    }
    lgkm_drain();
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        // rows 8g + qq (elements 0-3) and 8g + 4 + qq (4-7), iterate columns 16t + 4p4 .. +3
        const uint8_t* a0 = my0 + (s * 32 + 8 * g + qq) * XS + 2 * (16 * t) + 8 * p4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * XS));
        XF[8 * rd + s][t] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    lgkm_drain();
  }
  *reinterpret_cast<uint4*>(&bzero[w][16 * lane]) = make_uint4(0, 0, 0, 0);
  lgkm_drain();

  // ---- the wave's DMA of block kb (clamped: past the range it re-reads the range's last
  // block into the free slot, unused, so every step issues the same number of loads)
  const int64_t lda = a.lda;
  // ---- the strip ring.  A wave's slice of a block (16 rows x 512 columns) is 8 strips of 64
  // columns; strip k (2 KiB) sits at k * 2048, row r of it (128 B) at r * 128, logical 16-B
  // chunk c of the row at position c ^ sw(r): bank-conflict free for phase 1's row reads and
  // phase 2's transposed reads.  One DMA instruction moves half a strip (8 rows x 128 B; lane l:
  // row 8j + l / 8, position l % 8), so phase 2 hands a strip back as soon as its four column
  // tiles are read, and phase 1 waits for a block strip by strip.
  // Per-lane offsets from the block's first row at column c0: strip half j, a full strip or
  // one whose last 32 columns lie past cols (cols % 32 == 0; those lanes re-read the first 32)
  uint32_t vfull[2], vpart[2];
  auto voffs = [&](int nv, uint32_t (&vf)[2], uint32_t (&vp)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pr = 8 * j + (lane >> 3);     // row position in the strip
      const int rr = pr < nv ? pr : nv - 1;   // rows past the end re-read the last row (R = 0)
      const int c = (lane & 7) ^ sw(pr);
      const uint32_t rb = uint32_t(rr) * uint32_t(lda) * 2u;
      vf[j] = rb + uint32_t(c) * 16u;
      vp[j] = rb + uint32_t(c & 3) * 16u;
    }
  };
  voffs(PRB, vfull, vpart);
  struct Blk {
    const uint16_t* p;  // first row of the block (clamped into the range)
    int nv;             // valid rows
  };
  auto blk = [&](int kb) __attribute__((always_inline)) {
    const int kc = kb < kb1 ? kb : kblast;
    const int64_t r0 = int64_t(kc) * PRB;
    return Blk{A + r0 * lda, int(rows - r0 < PRB ? rows - r0 : PRB)};
  };
  // strip k of a block into a slot: 2 instructions.  Strips wholly past cols load columns
  // 0 .. 31 (finite data that meets X = 0; their G columns are never stored)
  auto dma_strip = [&](const Blk& b, const uint32_t (&vf)[2], const uint32_t (&vp)[2], int k, uint8_t* slot)
      __attribute__((always_inline)) {
    if constexpr (FULL) {
      // every strip of every block lies inside the rows: base = the block's first row at c0,
      // strip k at the immediate offset 128 k (k is a constant once the loops are unrolled)
      const uint16_t* base = b.p + c0;
      const uint32_t v1m = vf[1] - 1024u;
      uint8_t* d = slot + 2048 * k;
      switch (k) {
        case 0: dma_strip_off<0>(base, vf[0], v1m, d); break;
        case 1: dma_strip_off<128>(base, vf[0], v1m, d); break;
        case 2: dma_strip_off<256>(base, vf[0], v1m, d); break;
        case 3: dma_strip_off<384>(base, vf[0], v1m, d); break;
        case 4: dma_strip_off<512>(base, vf[0], v1m, d); break;
        case 5: dma_strip_off<640>(base, vf[0], v1m, d); break;
        case 6: dma_strip_off<768>(base, vf[0], v1m, d); break;
        default: dma_strip_off<896>(base, vf[0], v1m, d); break;
      }
    } else {
      const int cb = c0 + 64 * k;
      const bool full = cb + 64 <= cols;
      const uint16_t* base = b.p + (cb < cols ? cb : 0);
#pragma unroll
      for (int j = 0; j < 2; ++j) dma_row(base, full ? vf[j] : vp[j], slot + 2048 * k + 1024 * j);
    }
  };
  auto dma = [&](int kb, uint8_t* slot) __attribute__((always_inline)) {
    const Blk b = blk(kb);
    uint32_t vf[2], vp[2];
    voffs(b.nv, vf, vp);
#pragma unroll
    for (int k = 0; k < 8; ++k) dma_strip(b, vf, vp, k, slot);
  };
  // L2 prefetch of block kb: 4 B per lane into a per-wave sink nobody reads, a lane per 128-B
  // line; member h takes rows 8h .. 8h + 7 of the wave's slice (the pair shares the XCD's L2),
  // so the DMA of the block, pfd steps later, finds its lines on chip.  Always issued (pfd = 0
  // re-touches the block being loaded), so every wait counts the same loads
  const int pfd = batch.pfd;
  const uint32_t pfoff = uint32_t(c0 + 64 * (lane & 7) < cols ? c0 + 64 * (lane & 7) : 0) * 2u;
  const uint32_t pfv = uint32_t(lane >> 3) * uint32_t(lda) * 2u + pfoff;  // FULL: lane offset from row 8h
  auto pf = [&](int kb) __attribute__((always_inline)) {
    const int kc = kb < kb1 ? kb : kblast;
    if constexpr (FULL) {
      pf4_s(A + (int64_t(kc) * PRB + 8 * h) * lda, pfv, &sink[w][0]);
    } else {
      int64_t row = int64_t(kc) * PRB + 8 * h + (lane >> 3);
      row = row < rows ? row : rows - 1;
      pf4(reinterpret_cast<const uint8_t*>(A + row * lda) + pfoff, &sink[w][0]);
    }
  };
  // B of a block (16 rows x 32 iterates of half h = 16 x 64 B): one instruction of wave 0; the
  // other waves touch the same rows into their sink instead, so every wave counts one load
  const int brow = lane >> 2, bpiece = lane & 3;
  const uint32_t bv = uint32_t(brow * K + 8 * bpiece) * 2u;  // FULL: lane offset from the block's first B row
  auto dma_b = [&](int kb, uint8_t* bslot) __attribute__((always_inline)) {
    const int kc = kb < kb1 ? kb : kblast;
    if constexpr (FULL) {
      const uint16_t* sb = Bm + int64_t(kc) * PRB * K + PH * h;
      if (w == 0) dma16_s(sb, bv, bslot);
      else pf4_s(sb, bv, &sink[w][0]);
    } else {
      int64_t row = int64_t(kc) * PRB + brow;
      row = row < rows ? row : rows - 1;
      const uint16_t* src = Bm + row * K + PH * h + 8 * bpiece;
      if (w == 0) dma16(src, bslot);
      else pf4(src, &sink[w][0]);
    }
  };
  // vmcnt(n) alone (expcnt / lgkmcnt fields left free)
#define MPA_VMCNT(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (((n) >> 4) << 14) | 0x0F70)
  // strip k of the current block has landed once at most the loads issued after it are
  // pending: the rest of the block's strips (2 (7 - k)), its prefetch, and the next block's B,
  // 16 strip loads and prefetch (18).  k is a constant after unrolling: one wait survives
  auto wait_strip = [&](int k) __attribute__((always_inline)) {
    switch (k) {
      case 0: MPA_VMCNT(2 * 7 + 19); break;
      case 1: MPA_VMCNT(2 * 6 + 19); break;
      case 2: MPA_VMCNT(2 * 5 + 19); break;
      case 3: MPA_VMCNT(2 * 4 + 19); break;
      case 4: MPA_VMCNT(2 * 3 + 19); break;
      case 5: MPA_VMCNT(2 * 2 + 19); break;
      case 6: MPA_VMCNT(2 * 1 + 19); break;
      default: MPA_VMCNT(19); break;
    }
  };

  // G^T tiles of 32 iterates x 32 columns in a[16 ct .. 16 ct + 15] (mfma32): lane l column
  // l & 31, register r iterate (r & 3) + 8 (r >> 2) + 4 (l >> 5)
  g_zero();

  // step u issues block u + 2: B, its 8 strips (inside phase 2, as block u's strips are read),
  // then the prefetch of block u + 2 + pfd.  The prologue issues what steps -2 and -1 would
  // have, so every wait counts the same loads; blocks 2 .. pfd - 1, which no step prefetches,
  // go first (older than everything the waits count)
  for (int d = 2; d < pfd; ++d) pf(kb0 + d);
  dma_b(kb0, bring[0]);
  dma(kb0, my0);
  pf(kb0 + pfd);
  dma_b(kb0 + 1, bring[1]);
  dma(kb0 + 1, my1);
  pf(kb0 + 1 + pfd);

  // LDS offsets inside a slot: k-step s reads chunk 4 (s & 1) + g of row i of strip s / 2;
  // column tile ct reads chunks 2 (ct & 3), +1 of rows r0 and r0 + 4 of strip ct / 4
  // column tile ct (32 columns) of strip ct / 2 reads rows 8h + q (+4: +512 B) at chunk
  // 4 (ct & 1) + 2 cg + p4 / 2 (lane: h = l >> 5, cg = (l >> 4) & 1, q = qq, p4 = l & 3)
  int off1[2], off2[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) off1[s2] = i * 128 + ((4 * s2 + g) ^ sw(i)) * 16;
  {
    const int r0 = 8 * (lane >> 5) + qq, cg = (lane >> 4) & 1;
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) off2[c2] = r0 * 128 + ((4 * c2 + 2 * cg + (p4 >> 1)) ^ sw(r0)) * 16 + 8 * (p4 & 1);
  }

  // -I as the B operand of iterate tile t: lane (i, g) holds k = 8g .. 8g + 7 of column n = i
  bf16x8 NEGI[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) NEGI[t][j] = (8 * g + j == 16 * t + i) ? (__bf16)(-1.0f) : (__bf16)(0.0f);

  auto step = [&](int u, uint8_t* slot, uint8_t* bslot, f32x4 (&pt)[QW][2][64]) __attribute__((always_inline)) {
    // ---- phase 1: P_w[rows 4g + r][iterate 16 t + i].  Fragment reads run AD k-steps ahead
    // of the MFMAs, each strip's after its wait
    constexpr int AD = MPA_LSQP4_AD;
    wait_strip((AD - 1) / 2);  // the strips of the first AD k-steps (and B, older)
#if MPA_LSQP4_VACC
    // every wave starts its chain with the B MFMA: wave 0 DMA'd B, and its accumulators start
    // at -B (A operand: lane (i, g) = row i, iterates 8g .. 8g + 7 of the half, one 16-B read of
    // the row-major slot, against -I: exact, one nonzero product per output added to 0); the
    // other waves read a zero slot, so their chains start at 0 with no separate initialisation
    f32x4 p1[2];
    {
      const bf16x8 bfr = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
          (w == 0 ? bslot : &bzero[w][0]) + i * (PH * 2) + 16 * g));
      p1[0] = mfma_v0(bfr, NEGI[0]);
      p1[1] = mfma_v0(bfr, NEGI[1]);
    }
#else
    f32x4 p1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    if (w == 0) {
      // wave 0 DMA'd B: its accumulators start at -B, by one MFMA per iterate tile of the B rows
      // (A operand: lane (i, g) = row i, iterates 8g .. 8g + 7 of the half, one 16-B read of the
      // row-major slot) against -I (exact: one nonzero product per output, added to 0)
      const bf16x8 bfr = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(bslot + i * (PH * 2) + 16 * g));
      p1[0] = mfma(bfr, NEGI[0], p1[0]);
      p1[1] = mfma(bfr, NEGI[1], p1[1]);
    }
#endif
    {
    bf16x8 af[AD];
    auto rd1 = [&](int s) __attribute__((always_inline)) {
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(slot + off1[s & 1] + 2048 * (s >> 1)));
    };
#pragma unroll
    for (int s = 0; s < AD; ++s) af[s] = rd1(s);
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      __builtin_amdgcn_sched_barrier(0);
      if (s + AD < NKS && ((s + AD) & 1) == 0) wait_strip((s + AD) / 2);
#if MPA_LSQP4_PROBE & 4
      (void)af;
#elif MPA_LSQP4_VACC
      mfma_v(p1[0], af[s % AD], XF[s][0]);
      mfma_v(p1[1], af[s % AD], XF[s][1]);
#else
      p1[0] = mfma(af[s % AD], XF[s][0], p1[0]);
      p1[1] = mfma(af[s % AD], XF[s][1], p1[1]);
#endif
      if (s + AD < NKS) af[s % AD] = rd1(s + AD);
    }
    __builtin_amdgcn_sched_barrier(0);
#if MPA_LSQP4_VACC
    mfma_v_settle(p1[0], p1[1]);
#endif
    }
    // phase 2's column tiles in chunks of 2 = one strip (4 transposed reads), double-buffered:
    // the reads of chunk c + 1 go out between chunk c's MFMAs; chunk 0's before the reduce's
    // barrier (they read only this wave's slot)
    constexpr int CH = 2;
    s16x4 tb[2][CH][2];
    auto rd = [&](int c, s16x4 (&d)[CH][2]) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < CH; ++k) {  // tile 2c + k of strip c
        const uint8_t* src = slot + off2[k] + 2048 * c;
        d[k][0] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src));
        d[k][1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(src + 4 * 128));
      }
    };
    rd(0, tb[0]);
    // ---- reduce, one barrier: every wave sums the four partials (wave order; wave 0's carry
    // -B) into R in phase 1's accumulator layout (tile t, lane (i, g): rows 4g .. 4g + 3,
    // iterate 16t + i), splits it into bf16 hi + lo, and moves it into the 32x32x16 A operand
    // (lane l: iterate l & 31, rows 8(l >> 5) .. + 7) with one v_permlane16_swap per register
    // pair: swap(tile 0, tile 1) leaves 16-lane row k holding (t0 g0, t0 g1), (t1 g0, t1 g1),
    // (t0 g2, t0 g3), (t1 g2, t1 g3) for k = 0..3 -- exactly iterates 16(k & 1) + i, rows
    // 8(k >> 1) .. + 7
    bf16x8 RH, RL;
#if MPA_LSQP4_PROBE & 2
    if (true) {  // timing probe: no cross-wave exchange (own partial only, no barrier)
      f32x4 pv[2][QW];
      for (int t = 0; t < 2; ++t)
        for (int ww = 0; ww < QW; ++ww) pv[t][ww] = p1[t];
#else
    pt[w][0][lane] = p1[0];
    pt[w][1][lane] = p1[1];
    barrier();
    {
#endif
      const int64_t row0 = int64_t(kb0 + u) * PRB + 4 * g;
      const bool ragged = !FULL && int64_t(kb0 + u + 1) * PRB > rows;  // wave-uniform
#if !(MPA_LSQP4_PROBE & 2)
      f32x4 pv[2][QW];  // all eight reads in flight at once
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ww = 0; ww < QW; ++ww) pv[t][ww] = pt[ww][t][lane];
#endif
      uint32_t H[2][2], L[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 v = pv[t][0];
#pragma unroll
        for (int ww = 1; ww < QW; ++ww) v += pv[t][ww];
        if (ragged) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = row0 + r < rows ? v[r] : 0.f;  // rows past the end: R = 0
        }
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          // packed conversions (v_cvt_pk_bf16_f32, round to nearest even): hi of two rows at
          // once, back to fp32 by a shift / mask, lo of the remainders at once
          H[t][d] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{v[2 * d], v[2 * d + 1]}, bf16x2));
          const float h0 = __uint_as_float(H[t][d] << 16), h1 = __uint_as_float(H[t][d] & 0xffff0000u);
          L[t][d] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{v[2 * d] - h0, v[2 * d + 1] - h1}, bf16x2));
        }
      }
      uint32_t hx[2], hy[2], lx[2], ly[2];
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const auto sh = __builtin_amdgcn_permlane16_swap(H[0][d], H[1][d], false, false);
        const auto sl = __builtin_amdgcn_permlane16_swap(L[0][d], L[1][d], false, false);
        hx[d] = sh[0];
        hy[d] = sh[1];
        lx[d] = sl[0];
        ly[d] = sl[1];
      }
      RH = __builtin_bit_cast(bf16x8, make_uint4(hx[0], hx[1], hy[0], hy[1]));
      RL = __builtin_bit_cast(bf16x8, make_uint4(lx[0], lx[1], ly[0], ly[1]));
    }
    __builtin_amdgcn_sched_barrier(0);  // chunk 1's reads stay behind the reduce (registers)
    // ---- phase 2: G_w^T[it][col] += sum_row R^T[it][row] A[row][col] (hi, then lo); strip c of
    // the slot is refilled with block u + 2's once chunk c's MFMAs have consumed its reads
    dma_b(kb0 + u + 2, bslot);
    const Blk nb2 = blk(kb0 + u + 2);
    uint32_t vf[2] = {vfull[0], vfull[1]}, vp[2] = {vpart[0], vpart[1]};
    if (!FULL && nb2.nv < PRB) voffs(nb2.nv, vf, vp);
#pragma unroll
    for (int c = 0; c < NCT / CH; ++c) {
      lgkm_wait<0>();  // this chunk's reads, issued during the previous chunk's MFMAs
      __builtin_amdgcn_sched_barrier(0);
      if (c + 1 < NCT / CH) rd(c + 1, tb[(c + 1) & 1]);
      bf16x8 bt[CH];
#pragma unroll
      for (int k = 0; k < CH; ++k)
        bt[k] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(tb[c & 1][k][0], tb[c & 1][k][1], 0, 1, 2, 3, 4, 5, 6, 7));
      // each tile's lo MFMA right behind its hi MFMA: an XDL result read whole as SrcC by the NEXT
      // MFMA needs no wait states; with the other tile's MFMA between them it needs more than that
      // MFMA gives (the first version lost part of the hi products: 2e-4 errors)
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        mfma32(CH * c + k, RH, bt[k]);
        mfma32(CH * c + k, RL, bt[k]);
      }
      if (c + 1 < NCT / CH) {
#pragma unroll
        for (int j = 0; j < 2 * CH; ++j) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one LDS read
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#if !(MPA_LSQP4_PROBE & 1)  // timing probe 1: no strip DMAs in the loop (A stays stale in LDS)
      dma_strip(nb2, vf, vp, c, slot);
#endif
    }
    pf(kb0 + u + 2 + pfd);
  };
  for (int u = 0; u < nb; u += 2) {
    step(u, my0, bring[0], part[0]);
    if (u + 1 < nb) step(u + 1, my1, bring[1], part[1]);
  }
#undef MPA_VMCNT
  drain_vm();  // the trailing (unused) DMA pieces

  // ---- G over the row groups: fan-in-PF tree per (half, wave) of write-through partials
  const int nct = nks;                         // valid 32-column tiles
  const size_t wslab = size_t(4 * NCT) * 64;  // f32x4 units of one wave's partial
  f32x4* __restrict__ slab = static_cast<f32x4*>(a.slab) + (size_t(h) * kLsqpMaxGroups * QW + w) * wslab;
  const size_t qstride = size_t(QW) * wslab;  // between consecutive row groups
  uint32_t* ctr = a.ctr + (h * QW + w) * kLsqpCtrPerSlice;
  float* out = static_cast<float*>(a.out);
  // register group rg (G[ct][4 rg .. 4 rg + 3]) of tile ct: iterates 8 rg + 4 (l >> 5) .. + 3 of
  // column c0 + 32 ct + (l & 31)
  auto store_out = [&](int ct, int rg, const f32x4& v) __attribute__((always_inline)) {
    const int col = c0 + 32 * ct + (lane & 31);
    if (ct < nct && col < cols)
      *reinterpret_cast<f32x4*>(out + size_t(col) * K + PH * h + 8 * rg + 4 * (lane >> 5)) = v;
  };
  g_settle();
  auto quad = [](const f32x16& v, int rg) __attribute__((always_inline)) {
    return f32x4{v[4 * rg], v[4 * rg + 1], v[4 * rg + 2], v[4 * rg + 3]};
  };
  bool cx = false;
  if (ng == 1) {
    cx = disarmed(a.go, a.seq);
    if (!cx)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const f32x16 v = g_tile(ct);
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) store_out(ct, rg, quad(v, rg));
      }
  } else {
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const f32x16 v = g_tile(ct);
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) st_wt(slab + size_t(q) * qstride + (ct * 4 + rg) * 64 + lane, quad(v, rg));
    }
    unsigned idx = unsigned(q), count = unsigned(ng), stride = 1;
    int lvl_off = 0, lvl_cap = (kLsqpMaxGroups + PF - 1) / PF;
    for (;;) {
      drain_vm();
      const unsigned first = (idx / PF) * PF;
      const unsigned gsize = count - first < unsigned(PF) ? count - first : unsigned(PF);
      unsigned old = 0;
      if (lane == 0) {
        uint32_t* c = &ctr[lvl_off + int(idx / PF)];
        old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == gsize) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      old = __shfl(old, 0, 64);
      if (old + 1 != gsize) return;  // an earlier arriver of the group: the last one carries it
      const unsigned next = (count + PF - 1) / PF;
      if (next == 1) cx = disarmed(a.go, a.seq);
      const f32x4* src = slab + size_t(first) * stride * qstride;
#pragma unroll 4
      for (int j2 = 0; j2 < 4 * NCT; ++j2) {
        const int j = j2 * 64 + lane;
        f32x4 s = ld_wt(src + j);
        for (unsigned m = 1; m < gsize; ++m) s += ld_wt(src + size_t(m) * stride * qstride + j);
        if (next == 1) {
          if (!cx) store_out(j2 / 4, j2 % 4, s);
        } else {
          st_wt(slab + size_t(first) * stride * qstride + j, s);
        }
      }
      if (next == 1) break;
      idx /= PF;
      count = next;
      stride *= PF;
      lvl_off += lvl_cap;
      lvl_cap = (lvl_cap + PF - 1) / PF;
    }
  }
  // this slice of G is written: the task's last slice (2 halves x 4 waves) publishes
  drain_vm();
  if (lane == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain_vm();
    const unsigned old = __hip_atomic_fetch_add(&a.ctr[2 * 8 * kLsqpCtrPerSlice], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == unsigned(2 * QW)) {
      __hip_atomic_store(&a.ctr[2 * 8 * kLsqpCtrPerSlice], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!cx) publish_done(a.flag, a.seq);  // every slice read the same go word
    }
  }
}

}  // namespace

hipError_t launch_lsqp5(const LsqpBatch& a, hipStream_t s) {
  const int pairs = a.grp0[a.ntasks];
  if (pairs <= 0) return hipErrorInvalidValue;
  const int grid = (pairs + 7) / 8 * 16;
  bool full = true;
  for (int t = 0; t < a.ntasks; ++t) full = full && a.t[t].cols == kLsqpMaxCols && a.t[t].rows % PRB == 0;
  const bool armed = batch_armed(a);
  if (armed && full) hipLaunchKernelGGL((lsqp5_kernel<true, true>), dim3(grid), dim3(QT), 0, s, a);
  else if (armed) hipLaunchKernelGGL((lsqp5_kernel<true, false>), dim3(grid), dim3(QT), 0, s, a);
  else if (full) hipLaunchKernelGGL((lsqp5_kernel<false, true>), dim3(grid), dim3(QT), 0, s, a);
  else hipLaunchKernelGGL((lsqp5_kernel<false, false>), dim3(grid), dim3(QT), 0, s, a);
  return hipGetLastError();
}

}  // namespace mpa
