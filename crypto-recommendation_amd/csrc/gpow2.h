// gpow2.h — the reference's pow(x, 2), exactly as the process computes it.
//
// The reference squares every term of a distance and every norm component with
// glibc's pow (cust_vector.hpp:132, :149-150, :168-169; -O0 as shipped, so the
// call is real). glibc >= 2.28 pow (the optimized-routines algorithm) is not
// correctly rounded: its result before the final rounding is within ~0.011 ulp
// of x^2 (exp's 0.509-ulp bound plus the log's 1.3*2^-68 relative error scaled
// by |2 ln x|), so it differs from x*x (correctly rounded) only when x^2 lies
// within that distance of a rounding midpoint: ~0.085 % of general doubles,
// 1 ulp each. (x*x equals pow whenever x^2 is representable, e.g. x a
// difference of fp32 values with <= 26 significant bits.)
//
// gp_pow2_emul restates, operation for operation, the x86-64 __pow_fma variant
// that glibc 2.35's ifunc selects on FMA + AVX2 hosts (the disassembly's main
// path: log_inline, the y * log product, exp_inline and its specialcase, with
// the compiler's FMA contractions), for y = 2: a sign-free finite x goes
// through the tables of gpow2_tables.h (generated from this image's libm by
// tools/gen_pow_tables.py). Every step is one IEEE double add, multiply or fma
// in round-to-nearest, so host and device give the same bits.
// gp_sq(x) takes x*x when x^2 is provably not near a midpoint (|x| in
// [2^-40, 2^40], where the algorithm's error is <= 0.011 ulp, and x^2 more than
// 2^-6 ulp away from every midpoint) and the restatement otherwise (~3 % of
// general doubles, none of the exactly-representable squares; measured worst
// case of the algorithm: 0.0085 ulp, tests/pow2_check.cpp).
// Checked on the host against the process's real pow on ~2e9 inputs, near
// midpoints, ties, subnormals and the special ranges (tests/pow2_check.cpp); at
// run time, once per process, lshkm_ctx_create runs lshkm_pow_selfcheck()
// (pow2.hip) against the running process's pow and refuses to create a context
// (LSHKM_ERR_UNSUPPORTED) when they differ; the device path against host pow by
// tests/test_gpu_pow2.py.
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>

#include "gpow2_tables.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GP_HD __host__ __device__ inline
#define GP_HDM __host__ __device__ inline
static __device__ __constant__ const double gp_log_tab_d[128][3] = GP_LOG_TAB_INIT;
static __device__ __constant__ const uint64_t gp_exp_tab_d[256] = GP_EXP_TAB_INIT;
#else
#define GP_HD static inline
#define GP_HDM inline
#endif
static const double gp_log_tab_h[128][3] = GP_LOG_TAB_INIT;
static const uint64_t gp_exp_tab_h[256] = GP_EXP_TAB_INIT;

GP_HD uint64_t gp_bits(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint64_t)__double_as_longlong(x);
#else
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
#endif
}
GP_HD double gp_dbl(uint64_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __longlong_as_double((long long)u);
#else
    double x;
    memcpy(&x, &u, 8);
    return x;
#endif
}

// One table row; the device reads the __constant__ copy, the host its own.
#if defined(__HIP_DEVICE_COMPILE__)
#define GP_LOG_TAB gp_log_tab_d
#define GP_EXP_TAB gp_exp_tab_d
#else
#define GP_LOG_TAB gp_log_tab_h
#define GP_EXP_TAB gp_exp_tab_h
#endif
GP_HD void gp_log_row(int i, double* invc, double* logc, double* logctail) {
    *invc = GP_LOG_TAB[i][0];
    *logc = GP_LOG_TAB[i][1];
    *logctail = GP_LOG_TAB[i][2];
}
GP_HD uint64_t gp_exp_row(int i) { return GP_EXP_TAB[i]; }

// glibc 2.35 __pow_fma(x, 2.0), bit for bit (see the file comment).
GP_HD double gp_pow2_emul(double x) {
    const uint64_t ax = gp_bits(x) & 0x7fffffffffffffffull;
    // zero, inf, nan: pow returns x * x for y = 2 (its zeroinfnan(x) branch)
    if (ax == 0 || ax >= 0x7ff0000000000000ull) return x * x;
    // y = 2 is an even integer: a negative x gives sign_bias 0 and |x|
    uint64_t ix = ax;
    if ((ix >> 52) == 0) {                       // subnormal: normalise
        ix = gp_bits(x * 0x1p52) & 0x7fffffffffffffffull;
        ix -= 52ull << 52;
    }
    // ---- log_inline(ix): hi + tail ~ log(x) ----
    const uint64_t OFF = 0x3fe6955500000000ull;
    const uint64_t tmp = ix - OFF;
    const int i = (int)((tmp >> 45) & 127);
    const int k = (int)((int64_t)tmp >> 52);
    const uint64_t iz = ix - (tmp & (0xfffull << 52));
    const double z = gp_dbl(iz);
    const double kd = (double)k;
    double invc, logc, logctail;
    gp_log_row(i, &invc, &logc, &logctail);
    const double r = fma(z, invc, -1.0);
    const double t1 = fma(kd, GP_LN2HI, logc);
    const double lo1 = fma(kd, GP_LN2LO, logctail);
    const double ar = r * GP_A0;
    const double q12 = fma(r, GP_A2, GP_A1);
    const double q34 = fma(r, GP_A4, GP_A3);
    const double t2 = r + t1;
    const double ar2 = r * ar;
    const double tdf = t1 - t2;
    const double ar3 = r * ar2;
    const double lo3 = fma(ar, r, -ar2);
    const double lo2 = tdf + r;
    const double q56 = fma(r, GP_A6, GP_A5);
    const double hi = t2 + ar2;
    const double lo4a = t2 - hi;
    const double qa = fma(q56, ar2, q34);
    const double lo4 = lo4a + ar2;
    const double qq = fma(ar2, qa, q12);
    double s = lo1 + lo2;
    s = s + lo3;
    s = s + lo4;
    const double lo = fma(ar3, qq, s);
    const double ly = hi + lo;
    const double ltail = (hi - ly) + lo;
    // ---- y * log(x) as ehi + elo ----
    const double ehi = 2.0 * ly;
    const double elo = fma(2.0, ltail, fma(ly, 2.0, -ehi));
    // ---- exp_inline(ehi, elo, sign_bias = 0) ----
    const uint32_t abstop = (uint32_t)(gp_bits(ehi) >> 52) & 0x7ff;
    bool special = false;
    if (abstop - 0x3c9u >= 0x3fu) {
        if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + ehi;            // |ehi| < 2^-54
        if (abstop >= 0x409u) return (gp_bits(ehi) >> 63) ? 0.0 : gp_dbl(0x7ff0000000000000ull);  // uflow / oflow
        special = true;                                                   // 512 <= |ehi| < 1024
    }
    double kx = fma(ehi, GP_INVLN2N, GP_SHIFT);
    const uint64_t ki = gp_bits(kx);
    kx = kx - GP_SHIFT;
    double rr = fma(kx, GP_NEGLN2HIN, ehi);
    rr = fma(kx, GP_NEGLN2LON, rr);
    const uint64_t top = ki << 45;
    const int idx = 2 * (int)(ki & 127);
    const double tail = gp_dbl(gp_exp_row(idx));
    uint64_t sbits = gp_exp_row(idx + 1) + top;
    rr = elo + rr;
    const double p23 = fma(rr, GP_C3, GP_C2);
    const double tr = rr + tail;
    const double r2 = rr * rr;
    const double p45 = fma(rr, GP_C5, GP_C4);
    const double tt = fma(p23, r2, tr);
    const double r4 = r2 * r2;
    const double tm = fma(p45, r4, tt);
    if (!special) {
        const double scale = gp_dbl(sbits);
        return fma(tm, scale, scale);
    }
    // ---- specialcase(tm, sbits, ki) ----
    if ((ki & 0x80000000ull) == 0) {
        sbits -= 1009ull << 52;
        const double scale = gp_dbl(sbits);
        return fma(tm, scale, scale) * 0x1p1009;
    }
    sbits += 1022ull << 52;
    const double scale = gp_dbl(sbits);
    const double st = tm * scale;
    double y = scale + st;
    if (fabs(y) < 1.0) {
        const double one = y < 0.0 ? -1.0 : 1.0;
        const double lo5 = (scale - y) + st;
        const double hh = y + one;
        double v = (one - hh) + y;
        v = v + lo5;
        v = v + hh;
        y = v - one;
        if (y == 0.0) y = gp_dbl(sbits & 0x8000000000000000ull);
    }
    return y * 0x1p-1022;
}

// True when p = x*x is certainly the reference's pow(x, 2): the square is exact
// (x^2 - p = 0, and |x| >= 2^-460 so that a nonzero rest could not have
// underflowed to zero) or x is zero. pow returns a representable x^2 exactly
// (its error before rounding is far below half an ulp). Hot loops keep this as
// a per-row flag and send flagged rows to a gp_sq path.
GP_HD bool gp_sq_is(double x, double p) {
    return (fma(x, x, -p) == 0.0 && fabs(x) >= 0x1p-460) || x == 0.0;
}

// A sufficient test over a whole chain, without branches or fp64 work: x*x is
// pow(x, 2) whenever x has at most 26 significant bits (its square then fits
// the 53-bit significand: pow returns a representable x^2 exactly) and x^2 is
// not subnormal, so the chain ORs the low 32 bits of every x and checks the low
// 27 mantissa bits once (one v_or per square, two with v_or3). Zero, inf and
// nan have no such bits (their pow is x*x). TINY: the caller cannot rule out
// 0 < |x| < 2^-460 (a square near the subnormal range). hard() is false only
// if every square of the chain is certainly pow's value; a true hard() only
// costs a redo (x of 27 bits can still square exactly).
struct PwAcc {
    uint32_t lo = 0u;
    bool tiny = false;
    template <bool TINY>
    GP_HDM void add(double x) {
        lo |= (uint32_t)gp_bits(x);
        if (TINY) tiny = tiny | ((fabs(x) < 0x1p-460) & (x != 0.0));
    }
    GP_HDM bool hard() const { return (lo & 0x07FFFFFFu) != 0u || tiny; }
};

// True when p = x*x might not be pow(x, 2): |x| outside [2^-40, 2^40) (x != 0),
// x^2 just below a power of two, or x^2 within 2^-6 ulp of a rounding midpoint
// (see the file comment). The midpoint test without the ulp: with x^2 = p + e
// exactly, fma(e, K, p) for K = 32/31 (1 + 2^-40) rounds back to p iff |e K|
// <= ulp/2, i.e. |e| < 31/64 ulp: more than 1/64 ulp from the midpoint (an
// exact square, e = 0, always passes). ~9 VALU per square. The margin: 1/64
// = 0.0156 ulp against the algorithm's ~0.011-ulp bound; on 4e8 random squares
// no pow(x, 2) differs from x*x farther than 0.0086 ulp from a midpoint (the
// window was 2^-5 until round 6: twice the restatements).
GP_HD bool gp_sq_slow(double x, double p) {
    const double e = fma(x, x, -p);                        // x^2 = p + e exactly
    const double r = fma(e, 0x1.0842108422109p+0, p);      // K rounded up
    const double ax = fabs(x);
    const uint32_t hp = (uint32_t)(gp_bits(p) >> 32);
    const bool out = !(ax >= 0x1p-40 && ax < 0x1p40);      // nan too
    const bool pow2_below = (hp & 0xFFFFFu) == 0u && e < 0.0;   // ulp below p is ulp/2: restate
    return (r != p || out || pow2_below) && x != 0.0;
}

// pow(x, 2) as the reference computes it: x*x unless x^2 might sit near a
// rounding midpoint (see the file comment), then the restatement.
GP_HD double gp_sq(double x) {
    const double p = x * x;
    return gp_sq_slow(x, p) ? gp_pow2_emul(x) : p;
}

#if defined(__HIPCC__)
// NV squares per lane for a whole wave: p[j] = pow(x[j], 2). The few squares
// that need the restatement (~4 % of differences of fp32 values, ~6 % of
// general doubles) are packed from all lanes into lds (64 * NV doubles,
// wave-private; slots by ballot prefix counts, no scan) and evaluated 64 at a
// time, one per lane: a lane-per-chain gp_sq makes the wave run the
// restatement for nearly every term (a 64-lane wave almost always holds one
// such square). All 64 lanes must call it together.
// First the exact-square prefilter (PwAcc's test, wave-wide): when no value of
// any lane has more than 26 significant bits and none squares near the
// subnormal range, every x*x is pow's own value and nothing else runs (~2-4
// VALU per square instead of the midpoint test's ~9: fp32-grid rows, the
// reference's quantized inputs). TINY = false: the caller's values cannot lie
// in (0, 2^-460) (differences of fp32 values). EXSQ: the caller has proven every
// square exact (differences of a grid of <= 26 bits, data_grid_exact): x*x.
template <int NV, bool TINY = true, bool EXSQ = false>
__device__ inline void gp_sq_wave(const double (&x)[NV], double (&p)[NV], double* lds) {
    static_assert(NV <= 32, "lds holds 64 * NV doubles");
    if constexpr (EXSQ) {
#pragma unroll
        for (int j = 0; j < NV; j++) p[j] = __dmul_rn(x[j], x[j]);
        return;
    }
    uint32_t lo = 0u, hmin = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < NV; j++) {
        p[j] = __dmul_rn(x[j], x[j]);
        const uint64_t b = gp_bits(x[j]);
        lo |= (uint32_t)b;
        // |x| < 2^-460, zero excluded (0 - 1 wraps to the top); x with a zero
        // high word and low bits set fails the low-bits test anyway
        if (TINY) hmin = min(hmin, ((uint32_t)(b >> 32) & 0x7FFFFFFFu) - 1u);
    }
    if (__ballot((lo & 0x07FFFFFFu) != 0u || (TINY && hmin < 0x23300000u - 1u)) == 0ull) return;
    bool sl[NV];
    bool any = false;
#pragma unroll
    for (int j = 0; j < NV; j++) {
        sl[j] = gp_sq_slow(x[j], p[j]);
        any = any || sl[j];
    }
    if (__ballot(any) == 0ull) return;
    int pos[NV];
    int total = 0;
#pragma unroll
    for (int j = 0; j < NV; j++) {
        const unsigned long long m = __ballot(sl[j]);
        pos[j] = total + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        total += __popcll(m);
        if (sl[j]) lds[pos[j]] = x[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int lane = (int)__lane_id();
    for (int b = 0; b < total; b += 64)
        if (b + lane < total) lds[b + lane] = gp_pow2_emul(lds[b + lane]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < NV; j++)
        if (sl[j]) p[j] = lds[pos[j]];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");     // the next call's deposits come after these reads
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
#endif
