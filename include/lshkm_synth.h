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

/*
 * The "normal" generator (fp32 i.i.d. N(0,1) rows, full
 * mantissas): Irwin-Hall(12) -- the sum of twelve uniforms minus 6, mean 0,
 * variance exactly 1, the classic normal approximation (tails end at +-6) --
 * over 40-bit uniforms, so the sum is an integer of ~44 bits:
 *
 *   base = seed * 0x9E3779B97F4A7C15 + (row * d + col) * 12        (mod 2^64)
 *   S    = sum_{k<12} (splitmix64(base + k) >> 24)  -  6 * 2^40
 *   x    = (float)S * 2^-40          (one correctly rounded int64 -> fp32)
 *
 * Every value with |x| >= 2^-20 has a full 24-bit mantissa (the grid generator
 * above has <= 18 significant bits), so differences, squares and the f16
 * hi/lo splits are those of general fp32 data. Integer-only up to the one
 * rounding: gcc, numpy and the device give the same bits.
 */
LSHKM_HD float lshkm_synth_normal_value(uint64_t seed, uint64_t row, uint64_t d, uint64_t col) {
    const uint64_t base = seed * 0x9E3779B97F4A7C15ull + (row * d + col) * 12ull;
    int64_t s = -(int64_t)(6ull << 40);
    for (int k = 0; k < 12; k++) s += (int64_t)(lshkm_splitmix64(base + (uint64_t)k) >> 24);
    return (float)s * (1.0f / 1099511627776.0f);     /* 2^-40, exact */
}

#endif /* LSHKM_SYNTH_H */
