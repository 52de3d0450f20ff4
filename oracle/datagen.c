/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  C entry points of the Philox4x32-10 data layout
 * (philox.h) for the tests: a second, independent restatement beside lsq.py's numpy one.
 */
#include <stdint.h>

#include "philox.h"

void orc_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) { orc_philox4x32_10(ctr, key, out); }

void orc_gen_f32(uint64_t seed, uint32_t stream, uint64_t e0, int64_t count, float scale, float* out) {
  for (int64_t k = 0; k < count; ++k) out[k] = orc_unit_f32(orc_philox_word(seed, stream, e0 + (uint64_t)k)) * scale;
}

void orc_gen_f64(uint64_t seed, uint32_t stream, uint64_t e0, int64_t count, double scale, double* out) {
  for (int64_t k = 0; k < count; ++k) out[k] = (double)orc_unit_f32(orc_philox_word(seed, stream, e0 + (uint64_t)k)) * scale;
}
