// kmseg.h — the reference's sequential fp64 chain s_i = fl(s_{i-1} + x_i)
// (k_means, lib/clustering_phases/update.hpp:52-56 with addVectorToThis,
// cust_vector.hpp:177-184) evaluated in segments, bit for bit.
//
// While the partial sums stay inside one binade [2^E, 2^(E+1)) of one sign,
// they are integer multiples S of G = 2^(E-52) with 2^52 <= |S| < 2^53, and one
// step is S_i = S_{i-1} + m_i, m_i = x_i / G rounded to the nearest integer --
// an integer that does not depend on S_{i-1} unless x_i / G is a half-integer
// (a tie, rounded to the even S_i). A segment never continues through a tie,
// so it is summarised without its start value: the real first add s_a =
// fl(s_{a-1} + x_a), then the integer sum P of m_{a+1..b} and the range
// [lo, hi] of its prefix sums. The composition (one wave per chain) applies a
// segment in O(1): the real add, a check that s_a lies in the predicted binade
// with every S_a + prefix strictly inside it (|S| >= 2^52 + 1: a result at 2^E
// itself could have rounded in the finer grid below; |S| <= 2^53 - 1: 2^(E+1)
// belongs to the coarser grid above), and the exact add of P G. A segment
// whose check fails is walked with real adds -- the prediction (which binade
// each partial sum falls in, from approximate prefix sums) only decides where
// segments break, never the result.
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
#define KS_RECORDS 64
#endif
constexpr int KS_W = KS_WINDOW;    // member positions per window (pair = window x cluster)
constexpr int KS_R = KS_RECORDS;   // segment records per (pair, dim); more: the pair is walked
static_assert(KS_R <= 64, "one record per lane in the composition");

// One segment, as the composition applies it: s = fl(s + xa); the summary
// holds iff L <= s <= H (a range inside the predicted binade, folding in the
// prefix checks for every S_a); then s += d, exact: (S_a + P) G is a double of
// the same binade. Single-step segments: L = -inf, H = +inf, d = -0.0
// (s + -0.0 == s, signed zeros included). meta: bits 0-15 first offset a,
// 16-31 last offset b (in the window).
struct KsRec {
    double xa;
    double L, H;
    double d;          // P G
    uint64_t meta;     // 40 B
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
struct KsSeg {
    int key;           // 0: single-step segment
    int a, n;          // first offset, steps after the first
    int sh;            // 52 - E: x / G = ldexp(x, sh)
    double xa;
    double p, lo, hi;
};

KS_HD void ks_open(KsSeg& g, int key, int a, double xa) {
    g.key = key; g.a = a; g.n = 0; g.xa = xa;
    g.sh = 52 - ((key & 2047) - 1023);
    g.p = 0.0; g.lo = INFINITY; g.hi = -INFINITY;
}

// The step's integer m = x / G rounded to nearest by the 1.5 * 2^52 shifter;
// ok: |x / G| < 2^51 (false for inf / nan) and not a tie (|x / G - m| = 1/2,
// where the rounding would depend on the parity of S_{i-1}: the segment ends).
struct KsStep {
    double r;
    bool ok;
};
KS_HD KsStep ks_step_m(double x, int sh) {
    KsStep t;
    const double y = ldexp(x, sh);                    // exact (power-of-two scaling)
    t.r = (y + 0x1.8p52) - 0x1.8p52;
    t.ok = fabs(y) < 0x1p51 && fabs(y - t.r) != 0.5;
    return t;
}
KS_HD void ks_commit(KsSeg& g, const KsStep& t) {
    g.p += t.r;
    g.lo = fmin(g.lo, g.p);
    g.hi = fmax(g.hi, g.p);
    g.n++;
}

// Segmentation of one pair's positions: x at offset o, st the approximate
// partial sum after it. The segment continues while the predicted key holds
// and the step has a summary; otherwise the open segment is emitted and a new
// one starts at o (its first step is the real add of the composition).
// Branch-free except for the emit (a store): both outcomes are formed and
// selected, so lanes that continue and lanes that start a segment run the same
// instructions (the segment pass runs one lane per dimension).
template <typename Emit>
KS_HD void ks_feed(KsSeg& g, bool& open, double x, double st, int o, Emit&& emit) {
    const int key = ks_key(st);
    const KsStep t = ks_step_m(x, g.sh);
    const bool cont = open && key != 0 && key == g.key && t.ok;
    if (open && !cont) emit(g);
    const double p = g.p + t.r;
    g.p = cont ? p : 0.0;
    g.lo = cont ? fmin(g.lo, p) : INFINITY;
    g.hi = cont ? fmax(g.hi, p) : -INFINITY;
    g.n = cont ? g.n + 1 : 0;
    g.a = cont ? g.a : o;
    g.xa = cont ? g.xa : x;
    g.sh = cont ? g.sh : 52 - ((key & 2047) - 1023);
    g.key = cont ? g.key : key;
    open = true;
}

// What the segment pass stores (the same 40 B): the summary before its bounds
// are formed -- ks_finish forms them where the records are loaded (one lane per
// record there, so the per-step loop of the segment pass carries no ldexp /
// bound arithmetic on its divergent emit path). meta: a | b << 16 | key << 32.
struct KsRaw {
    double xa;
    double p, lo, hi;
    uint64_t meta;
};
KS_HD KsRaw ks_raw(const KsSeg& g) {
    KsRaw w;
    w.xa = g.xa; w.p = g.p; w.lo = g.lo; w.hi = g.hi;
    w.meta = (uint64_t)g.a | ((uint64_t)(g.a + g.n) << 16) | ((uint64_t)(uint32_t)g.key << 32);
    return w;
}

KS_HD KsRec ks_finish(const KsRaw& w) {
    KsRec r;
    r.xa = w.xa;
    r.meta = w.meta & 0xFFFFFFFFu;
    const int a = (int)(w.meta & 0xFFFFu), b = (int)((w.meta >> 16) & 0xFFFFu);
    const int key = (int)((w.meta >> 32) & 0xFFFu);
    if (b == a) {
        r.L = -INFINITY; r.H = INFINITY; r.d = -0.0;
        return r;
    }
    const int E = (key & 2047) - 1023;
    const bool neg = (key >> 11) & 1;
    double Lv, Hv;                                    // bounds on S_a (integers)
    if (!(fabs(w.lo) < 0x1p52 && fabs(w.hi) < 0x1p52)) { Lv = 1.0; Hv = 0.0; }
    else if (!neg) {      // 2^52 + 1 <= S_a + P <= 2^53 - 1 for every prefix P
        Lv = fmax(0x1p52 + 1.0 - w.lo, 0x1p52);
        Hv = fmin(0x1p53 - 1.0 - w.hi, 0x1p53 - 1.0);
    } else {              // -2^53 + 1 <= S_a + P <= -2^52 - 1
        Lv = fmax(-0x1p53 + 1.0 - w.lo, -0x1p53 + 1.0);
        Hv = fmin(-0x1p52 - 1.0 - w.hi, -0x1p52);
    }
    if (Lv > Hv) { r.L = INFINITY; r.H = -INFINITY; }
    else { r.L = ldexp(Lv, E - 52); r.H = ldexp(Hv, E - 52); }
    r.d = ldexp(w.p, E - 52);
    return r;
}
KS_HD KsRec ks_record(const KsSeg& g) { return ks_finish(ks_raw(g)); }

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
    s = KS_ADD(s, r.d);                               // exact
    return true;
}

}  // namespace lshkm
