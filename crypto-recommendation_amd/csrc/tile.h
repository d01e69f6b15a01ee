// tile.h — the split-f16 MFMA tile helpers shared by the fused hash+assign
// pass (fused.hip) and the standalone MFMA hash (hash_mfma.hip): operand
// types, the certification constants of DESIGN.md §4, EuclideanPhi's 32-bit
// arithmetic (euclidean_phi_gen.hpp:70-92) and the bucket division.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lshkm {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int FU_D = 128;                // dimension handled by this kernel
constexpr int FU_RS = FU_D + 8;          // f16 LDS row stride (elements) = 272 B

constexpr double FU_A1 = 1.25 * 0x1p-16;
// Hash tile of the persistent form: hi products of each 16-dim step in a fresh
// accumulator (<= 15 roundings), steps added in f32 (+7), + lo (+1): 23 * 2^-23
// = 0.72 * 2^-18 of sum|terms|; the split residuals and lo terms add < 0.25 *
// 2^-18 as in A1's derivation.
constexpr double FU_A1H = 1.25 * 0x1p-18;
constexpr double FU_A2 = 0x1p-24;
constexpr float FU_RANGE = 32768.f;

// phi % nb by multiply-high (Granlund-Montgomery round-up, 31-bit numerators):
// nb in [2, 2^31), l = ceil(log2 nb), m = floor(2^(31+l) / nb) + 1 < 2^32,
// q = (m * phi) >> (31 + l). nb == 1 -> 0; nb >= 2^31 -> phi (phi < 2^31).
struct BucketDiv {
    uint32_t m, nb;
    int sh, mode;           // mode 0: magic, 1: nb == 1, 2: nb > phi always
};
__host__ inline BucketDiv make_bucket_div(int64_t nb) {
    BucketDiv b{0u, 0u, 0, 0};
    if (nb <= 1) { b.mode = 1; return b; }
    if (nb >= (1ll << 31)) { b.mode = 2; return b; }
    int l = 0;
    while ((1ll << l) < nb) l++;
    b.m = (uint32_t)((((unsigned __int128)1 << (31 + l)) / (unsigned __int128)nb) + 1);
    b.nb = (uint32_t)nb;
    b.sh = l - 1;
    return b;
}

typedef float float2v __attribute__((ext_vector_type(2)));
constexpr double FU_SQRT_D = 11.313708498984761 * (1.0 + 0x1p-40);   // sqrt(128), rounded up

typedef _Float16 half2v __attribute__((ext_vector_type(2)));
// x - f32(h) in one v_fma_mix_f32 (x * 1 - h, the f16 operand widened exactly,
// one rounding: the same value as x - (float)h), h the low / high half of hp.
__device__ inline float resid_lo(float x, half2v hp) {
    float r;
    asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r) : "v"(x), "v"(hp));
    return r;
}
__device__ inline float resid_hi(float x, half2v hp) {
    float r;
    asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r) : "v"(x), "v"(hp));
    return r;
}

// EuclideanPhi arithmetic (euclidean_phi_gen.hpp:70-92) in 32-bit form, M =
// int(pow(2,32)-5) = 2^31-1 under g++. temp = (long)(h * r) is an int32 (the
// int product wraps), so ((temp % M) + M) % M needs only compares; the uint32
// sum hn wraps, and (hn % M + M) % M = hn % M for hn < 2^32.
constexpr uint32_t PHI_M = 2147483647u;
__device__ inline uint32_t phi_term(int32_t h, int32_t r) {
    int64_t v = (int32_t)((uint32_t)h * (uint32_t)r);    // in [-2^31, 2^31)
    if (v >= (int64_t)PHI_M) v -= PHI_M;
    if (v < 0) v += PHI_M;
    if (v < 0) v += PHI_M;                                 // only v = -2^31
    return (uint32_t)v;
}
__device__ inline uint32_t phi_final(uint32_t hn) {
    if (hn >= PHI_M) hn -= PHI_M;
    if (hn >= PHI_M) hn -= PHI_M;
    return hn;
}
// phi % nb (cust_hashtable.hpp:68); phi < 2^31
__device__ inline int32_t bucket_of(uint32_t ph, int64_t nb) {
    return nb <= 0xFFFFFFFFll ? (int32_t)(ph % (uint32_t)nb) : (int32_t)ph;
}
// Certified hashes have |h| < 2^22 and r in [0, 100] (euclidean_phi_gen.hpp:64;
// ProjTable::r_small), so h * r does not wrap, both operands fit 24 bits (one
// full-rate v_mul_i32_i24 instead of a quarter-rate v_mul_lo_u32) and
// ((temp % M) + M) % M is one select. Uncertified h are rewritten by the fix-up.
__device__ inline uint32_t phi_term_small(int32_t h, int32_t r) {
    const int32_t p = __mul24(h, r);
    return p < 0 ? (uint32_t)p + PHI_M : (uint32_t)p;
}
__device__ inline int32_t bucket_fast(uint32_t ph, const BucketDiv& b) {
    if (b.mode == 1) return 0;
    if (b.mode == 2) return (int32_t)ph;
    const uint32_t q = __umulhi(ph, b.m) >> b.sh;
    return (int32_t)(ph - q * b.nb);
}

// hi = f16(x) of 8 values; r = x - f32(hi) (one v_fma_mix each, exact) summed
// as r^2 into r2; LO: lo = f16(r) as well (the 3-product hash tile).
template <bool LO>
__device__ inline void split8_hi(const float* x, half8& hi, half8& lo, float2v& r2) {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        const half2v hp = {(_Float16)x[j], (_Float16)x[j + 1]};
        hi[j] = hp.x;
        hi[j + 1] = hp.y;
        const float2v r = {resid_lo(x[j], hp), resid_hi(x[j + 1], hp)};
        r2 = __builtin_elementwise_fma(r, r, r2);
        if (LO) {
            lo[j] = (_Float16)r.x;
            lo[j + 1] = (_Float16)r.y;
        }
    }
}

}  // namespace lshkm
