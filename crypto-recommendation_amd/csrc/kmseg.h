// kmseg.h — the reference's sequential fp64 chain s_i = fl(s_{i-1} + x_i)
// (k_means, lib/clustering_phases/update.hpp:52-56 with addVectorToThis,
// cust_vector.hpp:177-184) evaluated in segments, bit for bit.
//
// While the partial sums stay inside one binade [2^E, 2^(E+1)) of one sign,
// they are integer multiples S of G = 2^(E-52) with 2^52 <= |S| < 2^53, and one
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

#ifndef KS_WINDOW
#define KS_WINDOW 512
#endif
#ifndef KS_RECORDS
#define KS_RECORDS 32
#endif
constexpr int KS_W = KS_WINDOW;    // member positions per window (pair = window x cluster)
constexpr int KS_R = KS_RECORDS;   // segment records per (pair, dim); more: the pair is walked

// One segment, as the composition applies it: s = fl(s + xa); the summary
// holds iff L <= s <= H (a range inside the predicted binade, folding in the
// prefix checks for every S_a -- the union over both parities); then s += d0
// or d1 by the parity of S_a (the last significand bit of s). s + d is exact:
// (S_a + M) G is a double of the same binade. Single-step segments: L = -inf,
// H = +inf, d = -0.0 (s + -0.0 == s, signed zeros included). meta: bits 0-15
// first offset a, 16-31 last offset b (in the window).
struct KsRec {
    double xa;
    double L, H;
    double d0, d1;     // M G for an even / odd S_a
    uint64_t meta;     // 48 B: three 16-B loads
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

// Integer-valued doubles throughout: m_i and the prefix sums P are exact while
// |P| < 2^53; a segment whose prefix ever leaves that range has |lo| or |hi|
// >= 2^52 and can never pass its check, so rounding beyond it is harmless.
// par0 / par1: the parity of S_{i-1} in the even / odd S_a scenario.
struct KsSeg {
    int key;           // 0: single-step segment
    int a, n;          // first offset, steps after the first
    int par0, par1;
    double xa;
    double p0, p1, lo, hi;
};

KS_HD void ks_open(KsSeg& g, int key, int a, double xa) {
    g.key = key; g.a = a; g.n = 0; g.xa = xa;
    g.par0 = 0; g.par1 = 1;
    g.p0 = 0.0; g.p1 = 0.0; g.lo = INFINITY; g.hi = -INFINITY;
}

// The step's integer m, branch-free: r = x / G rounded to nearest-even by the
// 1.5 * 2^52 shifter (its last significand bit is r's parity); at a tie
// (|x / G - r| = 1/2) the reference rounds to the even S_i, so the scenario
// whose S_{i-1} is odd takes the other candidate 2 x / G - r. After a tie S_i
// is even in both scenarios.
struct KsStep {
    double r, alt;
    bool tie, ok;
    int pr;
};
KS_HD KsStep ks_step_m(double x, int key) {
    KsStep t;
    const int E = (key & 2047) - 1023;
    const double y = ldexp(x, 52 - E);                // exact (power-of-two scaling)
    t.ok = fabs(y) < 0x1p51;                           // false for inf / nan
    const double u = y + 0x1.8p52;
    t.r = u - 0x1.8p52;
    t.pr = (int)(ks_bits(u) & 1u);
    t.tie = fabs(y - t.r) == 0.5;
    t.alt = 2.0 * y - t.r;                            // exact: an integer next to r
    return t;
}
KS_HD void ks_commit(KsSeg& g, const KsStep& t) {
    const double m0 = (t.tie && g.par0) ? t.alt : t.r;
    const double m1 = (t.tie && g.par1) ? t.alt : t.r;
    g.par0 = t.tie ? 0 : (g.par0 ^ t.pr);
    g.par1 = t.tie ? 0 : (g.par1 ^ t.pr);
    g.p0 += m0;
    g.p1 += m1;
    g.lo = fmin(g.lo, fmin(g.p0, g.p1));
    g.hi = fmax(g.hi, fmax(g.p0, g.p1));
    g.n++;
}

// Segmentation of one pair's positions: x at offset o, st the approximate
// partial sum after it. The segment continues while the predicted key holds
// and the step has a summary; otherwise the open segment is emitted and a new
// one starts at o (its first step is the real add of the composition).
template <typename Emit>
KS_HD void ks_feed(KsSeg& g, bool& open, double x, double st, int o, Emit&& emit) {
    const int key = ks_key(st);
    const KsStep t = ks_step_m(x, g.key);
    if (open && key != 0 && key == g.key && t.ok) {
        ks_commit(g, t);
        return;
    }
    if (open) emit(g);
    ks_open(g, key, o, x);
    open = true;
}

KS_HD KsRec ks_record(const KsSeg& g) {
    KsRec r;
    r.xa = g.xa;
    r.meta = (uint64_t)g.a | ((uint64_t)(g.a + g.n) << 16);
    if (g.n == 0) {
        r.L = -INFINITY; r.H = INFINITY; r.d0 = -0.0; r.d1 = -0.0;
        return r;
    }
    const int E = (g.key & 2047) - 1023;
    const bool neg = (g.key >> 11) & 1;
    double Lv, Hv;                                    // bounds on S_a (integers)
    if (!(fabs(g.lo) < 0x1p52 && fabs(g.hi) < 0x1p52)) { Lv = 1.0; Hv = 0.0; }
    else if (!neg) {      // 2^52 + 1 <= S_a + P <= 2^53 - 1 for every prefix P
        Lv = fmax(0x1p52 + 1.0 - g.lo, 0x1p52);
        Hv = fmin(0x1p53 - 1.0 - g.hi, 0x1p53 - 1.0);
    } else {              // -2^53 + 1 <= S_a + P <= -2^52 - 1
        Lv = fmax(-0x1p53 + 1.0 - g.lo, -0x1p53 + 1.0);
        Hv = fmin(-0x1p52 - 1.0 - g.hi, -0x1p52);
    }
    if (Lv > Hv) { r.L = INFINITY; r.H = -INFINITY; }
    else { r.L = ldexp(Lv, E - 52); r.H = ldexp(Hv, E - 52); }
    r.d0 = ldexp(g.p0, E - 52);
    r.d1 = ldexp(g.p1, E - 52);
    return r;
}

KS_HD int ks_rec_a(const KsRec& r) { return (int)(r.meta & 0xFFFFu); }
KS_HD int ks_rec_b(const KsRec& r) { return (int)((r.meta >> 16) & 0xFFFFu); }

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
    if (!(s >= r.L && s <= r.H)) return false;        // nan: false
    s = KS_ADD(s, (ks_bits(s) & 1u) ? r.d1 : r.d0);  // exact
    return true;
}

}  // namespace lshkm
