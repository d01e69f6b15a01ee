// kmseg.h — the reference's sequential fp64 chain s_i = fl(s_{i-1} + x_i)
// (k_means, lib/clustering_phases/update.hpp:52-56 with addVectorToThis,
// cust_vector.hpp:177-184) evaluated in segments, bit for bit.
//
// While the partial sums stay inside one binade [2^E, 2^(E+1)) of one sign,
// they are integer multiples S of G = 2^(E-52) with 2^52 < |S| < 2^53, and one
// step is S_i = S_{i-1} + m_i, m_i = x_i / G rounded to the nearest integer
// (ties to the even S_i) -- an integer that does not depend on S_{i-1} except
// through its parity at a tie. A segment [a, b] is therefore summarised
// without its start value: the real first add s_a = fl(s_{a-1} + x_a), then
// for both parities of S_a the integer sum M of m_{a+1..b} and the range
// [lo, hi] of its prefix sums. The composition (one lane per chain) applies a
// segment in O(1): the real add, a check that s_a lies in the predicted
// binade, and a check that every S_a + prefix stays strictly inside it
// (|S| >= 2^52 + 1: a result at 2^E itself could have rounded in the finer
// grid below; |S| <= 2^53 - 1: 2^(E+1) belongs to the coarser grid above).
// A segment whose checks fail is walked with real adds -- the prediction
// (which binade each partial sum falls in, from approximate prefix sums) only
// decides where segments break, never the result.
//
// Used by update.hip's segmented k-means update (fp64 rows) and checked on the
// host against the plain chain by tests/kmseg_check.cpp.
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIPCC__)
#define KS_HD __host__ __device__ inline
#else
#define KS_HD static inline
#endif

namespace lshkm {

constexpr int KS_W = 512;          // member positions per window (pair = window x cluster)
constexpr int KS_R = 32;           // segment records per (pair, dim); more: the pair is walked

// One segment. meta: bits 0-15 dM = M1 - M0 (int16), 16-27 biased exponent
// (0: a single real add, no summary), bit 28 negative, 32-41 first offset a,
// 42-51 last offset b (in the window).
struct KsRec {
    double xa;
    int64_t m0;        // M for an even S_a
    int64_t lo, hi;    // prefix-sum range over both parities
    uint64_t meta;
    uint64_t pad;      // 48 B: three 16-B loads
};

KS_HD uint64_t ks_bits(double v) {
    uint64_t b;
    memcpy(&b, &v, 8);
    return b;
}

// key of a partial sum: biased exponent | sign << 11; 0 where no summary
// applies (zero / subnormal-adjacent, inf / nan, or near the top of the range)
KS_HD int ks_key(double s) {
    const uint64_t b = ks_bits(s);
    const int be = (int)((b >> 52) & 2047u);
    if (be < 24 || be > 2040) return 0;
    return be | (int)((b >> 63) << 11);
}

struct KsSeg {
    int key;           // 0: single-step segment
    int a, n;          // first offset, steps after the first
    double xa;
    int64_t p0, p1, lo, hi;
};

KS_HD void ks_open(KsSeg& g, int key, int a, double xa) {
    g.key = key; g.a = a; g.n = 0; g.xa = xa;
    g.p0 = 0; g.p1 = 0; g.lo = 0; g.hi = 0;
}

// One step x after the segment's first: false if x / G is not a usable integer
// candidate (|x / G| >= 2^54, inf / nan) -- the caller then breaks the segment.
KS_HD bool ks_step(KsSeg& g, double x) {
    const int E = (g.key & 2047) - 1023;
    const double y = ldexp(x, 52 - E);                // exact (power-of-two scaling)
    const double a = fabs(y);
    if (!(a < 0x1p54)) return false;
    const double na = floor(a);
    const double fa = a - na;                         // exact: a >= 0
    const int64_t ni = (int64_t)na;
    const bool neg = y < 0.0;
    const int64_t c_lo = neg ? -ni : ni;              // toward zero
    const int64_t c_hi = neg ? -ni - 1 : ni + 1;      // away from zero
    int64_t m0, m1;
    if (fa < 0.5) { m0 = c_lo; m1 = c_lo; }
    else if (fa > 0.5) { m0 = c_hi; m1 = c_hi; }
    else {                                            // tie: the candidate giving an even S
        m0 = ((g.p0 + c_lo) & 1) == 0 ? c_lo : c_hi;          // S_a even
        m1 = ((g.p1 + 1 + c_lo) & 1) == 0 ? c_lo : c_hi;      // S_a odd
    }
    g.p0 += m0;
    g.p1 += m1;
    const int64_t mn = g.p0 < g.p1 ? g.p0 : g.p1, mx = g.p0 < g.p1 ? g.p1 : g.p0;
    if (g.n == 0) { g.lo = mn; g.hi = mx; }
    else {
        g.lo = mn < g.lo ? mn : g.lo;
        g.hi = mx > g.hi ? mx : g.hi;
    }
    g.n++;
    return true;
}

// Segmentation of one pair's positions: x at offset o, st the approximate
// partial sum after it. The segment continues while the predicted key holds
// and the step has a summary; otherwise the open segment is emitted and a new
// one starts at o (its first step is the real add of the composition).
template <typename Emit>
KS_HD void ks_feed(KsSeg& g, bool& open, double x, double st, int o, Emit&& emit) {
    const int key = ks_key(st);
    if (open && key != 0 && key == g.key && ks_step(g, x)) return;
    if (open) emit(g);
    ks_open(g, key, o, x);
    open = true;
}

KS_HD KsRec ks_record(const KsSeg& g) {
    KsRec r;
    r.xa = g.xa;
    r.m0 = g.p0;
    r.lo = g.lo;
    r.hi = g.hi;
    const int64_t dm = g.p1 - g.p0;                   // |dm| <= number of ties < KS_W
    const int be = g.n ? (g.key & 2047) : 0;
    r.pad = 0;
    r.meta = (uint64_t)(uint16_t)(int16_t)dm | ((uint64_t)be << 16) | ((uint64_t)((g.key >> 11) & 1) << 28) |
             ((uint64_t)g.a << 32) | ((uint64_t)(g.a + g.n) << 42);
    return r;
}

KS_HD int ks_rec_a(const KsRec& r) { return (int)((r.meta >> 32) & 1023u); }
KS_HD int ks_rec_b(const KsRec& r) { return (int)((r.meta >> 42) & 1023u); }

// Apply a record to the running sum s (the real first add included). false:
// the summary does not apply -- s holds fl(s_{a-1} + x_a) and the caller adds
// positions a+1 .. b with real adds.
#if defined(__HIP_DEVICE_COMPILE__)
#define KS_ADD(a, b) __dadd_rn((a), (b))
#else
#define KS_ADD(a, b) ((a) + (b))
#endif
KS_HD bool ks_apply(double& s, const KsRec& r) {
    s = KS_ADD(s, r.xa);
    const int be = (int)((r.meta >> 16) & 2047u);
    if (be == 0) return true;                         // single step
    const uint64_t b = ks_bits(s);
    const int neg = (int)((r.meta >> 28) & 1u);
    if ((int)((b >> 52) & 2047u) != be || (int)(b >> 63) != neg) return false;
    const int E = be - 1023;
    const int64_t S = (int64_t)ldexp(s, 52 - E);      // exact: |S| in [2^52, 2^53)
    const int64_t dm = (int64_t)(int16_t)(uint16_t)(r.meta & 0xFFFFu);
    const int64_t M = (S & 1) ? r.m0 + dm : r.m0;
    constexpr int64_t B0 = (int64_t)1 << 52, B1 = (int64_t)1 << 53;
    const bool ok = neg ? (S + r.hi <= -B0 - 1 && S + r.lo >= -B1 + 1) : (S + r.lo >= B0 + 1 && S + r.hi <= B1 - 1);
    if (!ok) return false;
    s = ldexp((double)(S + M), E - 52);               // exact: |S + M| < 2^53
    return true;
}

}  // namespace lshkm
