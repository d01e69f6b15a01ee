/*
 * lshkm_synth.h — the synthetic point generator shared by the bench, the
 * tests, the CPU oracle and the reference harness.
 *
 * Integer-only, so every producer (gcc host code, numpy, a gfx950 kernel)
 * yields bit-identical fp32 values:
 *
 *   key = seed * 0x9E3779B97F4A7C15 + (row * d + col)     (mod 2^64)
 *   z   = splitmix64(key)
 *   S   = sum of the four 16-bit chunks of z  - 131070     (Irwin–Hall(4))
 *   x   = S * 2^-15                                       (exact in fp32)
 *
 * x is symmetric, bell-shaped (std ≈ 1.155), and exactly representable in
 * fp32 — the same storage contract as the reference's CSV doubles read from
 * fp32-valued data. It is synthetic data, not a claim about
 * real inputs.
 */
#ifndef LSHKM_SYNTH_H
#define LSHKM_SYNTH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define LSHKM_HD __host__ __device__ inline
#else
#define LSHKM_HD static inline
#endif

LSHKM_HD uint64_t lshkm_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

LSHKM_HD float lshkm_synth_value(uint64_t seed, uint64_t row, uint64_t d, uint64_t col) {
    uint64_t z = lshkm_splitmix64(seed * 0x9E3779B97F4A7C15ull + row * d + col);
    int32_t s = (int32_t)(z & 0xFFFF) + (int32_t)((z >> 16) & 0xFFFF) +
                (int32_t)((z >> 32) & 0xFFFF) + (int32_t)(z >> 48) - 131070;
    return (float)s * (1.0f / 32768.0f);
}

#endif /* LSHKM_SYNTH_H */
