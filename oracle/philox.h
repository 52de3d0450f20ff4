/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 * Philox4x32-10 counter-based RNG (Salmon, Moraes, Dror, Shaw, "Parallel random numbers:
 * as easy as 1, 2, 3", SC'11; the Random123 library's published algorithm), and the
 * synthetic least-squares data layout of the MI355X build.  The
 * reference has no data generator (its workers sleep: examples/iterative_example.jl:74),
 * so this layout is the build's own; the product's device generator
 * (mpistragglers.jl_amd/csrc/datagen.hip) must match it bit for bit.
 */
#ifndef MPA_ORACLE_PHILOX_H
#define MPA_ORACLE_PHILOX_H
#include <stdint.h>

static inline void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* 32-bit word for element e of stream s: counter (e/4 lo, e/4 hi, s, 0), word e%4 */
static inline uint32_t orc_philox_word(uint64_t seed, uint32_t stream, uint64_t e) {
  uint64_t q = e >> 2;
  uint32_t ctr[4] = {(uint32_t)q, (uint32_t)(q >> 32), stream, 0u};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  orc_philox4x32_10(ctr, key, o);
  return o[e & 3];
}

/* uniform in [-1, 1) on a 2^-23 grid: exact in fp32, fp64 and (after RNE) bf16 */
static inline float orc_unit_f32(uint32_t w) {
  return (float)((int32_t)(w >> 8) - 8388608) * (1.0f / 8388608.0f);
}
#endif
