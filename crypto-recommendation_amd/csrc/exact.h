// exact.h — the reference's point-to-centroid distances in its exact
// operation order, for the device paths that need the value itself.
//   euclideanDistance  lib/data_structures/cust_vector.hpp:124-136
//     sqrt(sum_j pow(x_j - c_j, 2)), fp64, j ascending
//   cosineDistance     lib/data_structures/cust_vector.hpp:139-155
//     1 - (long double) inner product / (sqrt(sum x^2) * sqrt(sum c^2))
// `this` is the point x (fp32 or fp64 values), `in` the centroid c (fp64).
// pow(v, 2) is gp_sq(v) (gpow2.h): glibc's own result, bit for bit. No FMA
// contraction.
#pragma once
#include "softx87.h"
#include "gpow2.h"

// pow(v, 2) of a value stored as T: an fp32 value squares exactly in fp64
// (48 significant bits, no underflow), so only fp64 values need gp_sq.
template <typename T>
__device__ inline double sq_of(double v) {
    if constexpr (sizeof(T) == 4) return __dmul_rn(v, v);
    else return gp_sq(v);
}

template <typename T>
__device__ inline double exact_euclid(const T* __restrict__ x, const double* __restrict__ c, int d) {
    double acc = 0.0;
    for (int j = 0; j < d; j++) {
        const double df = __dsub_rn((double)x[j], c[j]);
        acc = __dadd_rn(acc, gp_sq(df));
    }
    return sqrt(acc);
}

// double(ip / (long double)denom) for denom = sqrt(.) * sqrt(.) >= +0, with
// x87's results for a zero denominator (a zero vector): 0/0 is the default
// NaN "real indefinite" (sign set: 0xFFF8... as a double), x/0 = +-inf.
__device__ inline double x87_quot(sx80 ip, double denom) {
    if (denom == 0.0) {
        if (ip.m == 0) return __longlong_as_double((long long)0xFFF8000000000000ull);
        return ip.s ? -__builtin_inf() : __builtin_inf();
    }
    return sx_to_double(sx_div(ip, sx_from_double(denom)));
}

// 1 - q as SSE subsd computes it: a NaN q comes back unchanged.
__device__ inline double one_minus(double q) { return q != q ? q : __dsub_rn(1.0, q); }

// The soft-x87 form: every inner-product add emulated (~150 integer ops each).
template <typename T, typename U>
__device__ inline double exact_cosine_x87_soft(const T* __restrict__ x, const U* __restrict__ c, int d) {
    sx80 ip = sx_zero();
    double a = 0.0, b = 0.0;
    for (int j = 0; j < d; j++) {
        const double xj = (double)x[j], cj = (double)c[j];
        ip = sx_add_double(ip, __dmul_rn(xj, cj));
        a = __dadd_rn(a, sq_of<T>(xj));
        b = __dadd_rn(b, sq_of<U>(cj));
    }
    return one_minus(x87_quot(ip, __dmul_rn(sqrt(a), sqrt(b))));
}

// The reference's cosine distance exactly: the x87 inner-product chain carried
// as a double-double (softx87.h X87dd, ~30 fp64 ops per add, checked against
// real long double on the host), the soft FADD only past a sum X87dd does not
// decide (X87acc).
// xa / cb as cosine_interval's.
template <typename T, typename U>
__device__ inline double exact_cosine_x87(const T* __restrict__ x, const U* __restrict__ c, int d, double xa = -1.0,
                                          double cb = -1.0) {
    X87acc ip;
    ip.init();
    double a = 0.0, b = 0.0;
    const bool fa = xa < 0.0, fb = cb < 0.0;
    for (int j = 0; j < d; j++) {
        const double xj = (double)x[j], cj = (double)c[j];
        ip.add(__dmul_rn(xj, cj));
        if (fa) a = __dadd_rn(a, sq_of<T>(xj));
        if (fb) b = __dadd_rn(b, sq_of<U>(cj));
    }
    if (!fa) a = xa;
    if (!fb) b = cb;
    return one_minus(x87_quot(ip.value(), __dmul_rn(sqrt(a), sqrt(b))));
}

// exact_cosine_x87 lane per row with the next 8 terms' loads in flight while
// the current 8 are chained (one lane's chain is ~25 dependent fp64 operations
// per term; a load round trip per term made a lone row's chain ~45 us at
// d = 100). VEC: fp32 row and fp64 centroid rows 16-B aligned with d % 8 == 0
// (vector loads); otherwise element loads, the last chunk partial.
// xa / cb as cosine_interval's (precomputed sums of squares, else < 0).
template <bool VEC, typename T, typename U>
__device__ inline double exact_cosine_x87_pf(const T* __restrict__ x, const U* __restrict__ c, int d, double xa = -1.0,
                                             double cb = -1.0) {
    constexpr int B = 8;
    X87acc ip;
    ip.init();
    double a = 0.0, b = 0.0;
    const bool fa = xa < 0.0, fb = cb < 0.0;
    T xn[B];
    U cn[B];
    auto load = [&](int j0) {
        if constexpr (VEC) {
#pragma unroll
            for (int t = 0; t < 2; t++) {
                const float4 v = *reinterpret_cast<const float4*>(x + j0 + 4 * t);
                xn[4 * t] = v.x; xn[4 * t + 1] = v.y; xn[4 * t + 2] = v.z; xn[4 * t + 3] = v.w;
            }
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const double2 v = *reinterpret_cast<const double2*>(c + j0 + 2 * t);
                cn[2 * t] = v.x; cn[2 * t + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int t = 0; t < B; t++)
                if (j0 + t < d) { xn[t] = x[j0 + t]; cn[t] = c[j0 + t]; }
        }
    };
    load(0);
    for (int j0 = 0; j0 < d; j0 += B) {
        T xs[B];
        U cs[B];
#pragma unroll
        for (int t = 0; t < B; t++) { xs[t] = xn[t]; cs[t] = cn[t]; }
        if (j0 + B < d) load(j0 + B);
#pragma unroll
        for (int t = 0; t < B; t++) {
            if (!VEC && j0 + t >= d) break;
            const double xj = (double)xs[t], cj = (double)cs[t];
            ip.add(__dmul_rn(xj, cj));
            if (fa) a = __dadd_rn(a, sq_of<T>(xj));
            if (fb) b = __dadd_rn(b, sq_of<U>(cj));
        }
    }
    if (!fa) a = xa;
    if (!fb) b = cb;
    return one_minus(x87_quot(ip.value(), __dmul_rn(sqrt(a), sqrt(b))));
}

// The reference's euclidean distance lane per row with the next 8 terms' loads
// in flight (the pow fix-up list of the hi-only pass; VEC as above).
template <bool VEC, typename T, typename U>
__device__ inline double exact_euclid_pf(const T* __restrict__ x, const U* __restrict__ c, int d) {
    constexpr int B = 8;
    double acc = 0.0;
    T xn[B];
    U cn[B];
    auto load = [&](int j0) {
        if constexpr (VEC) {
#pragma unroll
            for (int t = 0; t < 2; t++) {
                const float4 v = *reinterpret_cast<const float4*>(x + j0 + 4 * t);
                xn[4 * t] = v.x; xn[4 * t + 1] = v.y; xn[4 * t + 2] = v.z; xn[4 * t + 3] = v.w;
            }
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const double2 v = *reinterpret_cast<const double2*>(c + j0 + 2 * t);
                cn[2 * t] = v.x; cn[2 * t + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int t = 0; t < B; t++)
                if (j0 + t < d) { xn[t] = x[j0 + t]; cn[t] = c[j0 + t]; }
        }
    };
    load(0);
    for (int j0 = 0; j0 < d; j0 += B) {
        T xs[B];
        U cs[B];
#pragma unroll
        for (int t = 0; t < B; t++) { xs[t] = xn[t]; cs[t] = cn[t]; }
        if (j0 + B < d) load(j0 + B);
#pragma unroll
        for (int t = 0; t < B; t++) {
            if (!VEC && j0 + t >= d) break;
            acc = __dadd_rn(acc, gp_sq(__dsub_rn((double)xs[t], (double)cs[t])));
        }
    }
    return sqrt(acc);
}

// The fix-up chains above with the whole wave in step (every lane calls them;
// a lane without a row repeats another's): each 8 terms' squares go through
// gp_sq_wave (sq: wave-private LDS), so the wave evaluates
// glibc's restatement for the few squares that need it in one batch instead of
// serialising one lane's restatement after another (a wave of lane chains
// holds one such square in nearly every term). sq: 64 * 8 doubles (euclidean,
// cosine on fp32 rows) or 64 * 16 (cosine on fp64 rows).
template <bool VEC, typename T, typename U>
__device__ inline void pf_load8(const T* __restrict__ x, const U* __restrict__ c, int j0, int d, T (&xn)[8],
                                U (&cn)[8]) {
    if constexpr (VEC) {
#pragma unroll
        for (int t = 0; t < 2; t++) {
            const float4 v = *reinterpret_cast<const float4*>(x + j0 + 4 * t);
            xn[4 * t] = v.x; xn[4 * t + 1] = v.y; xn[4 * t + 2] = v.z; xn[4 * t + 3] = v.w;
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const double2 v = *reinterpret_cast<const double2*>(c + j0 + 2 * t);
            cn[2 * t] = v.x; cn[2 * t + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int t = 0; t < 8; t++) {
            xn[t] = j0 + t < d ? x[j0 + t] : (T)0;
            cn[t] = j0 + t < d ? c[j0 + t] : (U)0;
        }
    }
}

template <bool VEC, typename T, typename U>
__device__ inline double exact_euclid_wave(const T* __restrict__ x, const U* __restrict__ c, int d, double* sq) {
    double acc = 0.0;
    T xn[8];
    U cn[8];
    pf_load8<VEC>(x, c, 0, d, xn, cn);
    for (int j0 = 0; j0 < d; j0 += 8) {
        double df[8], p[8];
#pragma unroll
        for (int t = 0; t < 8; t++) df[t] = __dsub_rn((double)xn[t], (double)cn[t]);
        if (j0 + 8 < d) pf_load8<VEC>(x, c, j0 + 8, d, xn, cn);
        gp_sq_wave<8>(df, p, sq);
#pragma unroll
        for (int t = 0; t < 8; t++) {
            if (!VEC && j0 + t >= d) break;
            acc = __dadd_rn(acc, p[t]);
        }
    }
    return sqrt(acc);
}

template <bool VEC, typename T, typename U>
__device__ inline double exact_cosine_x87_wave(const T* __restrict__ x, const U* __restrict__ c, int d, double* sq) {
    static_assert(sizeof(U) == 8, "fp64 centroids");
    constexpr int NS = sizeof(T) == 8 ? 16 : 8;         // squares through gp_sq_wave per 8 terms
    X87acc ip;
    ip.init();
    double a = 0.0, b = 0.0;
    T xn[8];
    U cn[8];
    pf_load8<VEC>(x, c, 0, d, xn, cn);
    for (int j0 = 0; j0 < d; j0 += 8) {
        double xv[8], cv[8], v[NS], p[NS];
#pragma unroll
        for (int t = 0; t < 8; t++) {
            xv[t] = (double)xn[t];
            cv[t] = (double)cn[t];
            v[t] = cv[t];
            if constexpr (NS == 16) v[8 + t] = xv[t];
        }
        if (j0 + 8 < d) pf_load8<VEC>(x, c, j0 + 8, d, xn, cn);
        gp_sq_wave<NS>(v, p, sq);
#pragma unroll
        for (int t = 0; t < 8; t++) {
            if (!VEC && j0 + t >= d) break;
            ip.add(__dmul_rn(xv[t], cv[t]));
            a = __dadd_rn(a, NS == 16 ? p[8 + t] : __dmul_rn(xv[t], xv[t]));
            b = __dadd_rn(b, p[t]);
        }
    }
    return one_minus(x87_quot(ip.value(), __dmul_rn(sqrt(a), sqrt(b))));
}

// fp32 rows of d % 16 == 0 (16-B aligned rows)
__device__ inline double exact_cosine_x87_b16(const float* __restrict__ x, const double* __restrict__ c, int d) {
    return exact_cosine_x87_pf<true>(x, c, d);
}

// Certified fast form of the x87 inner product's quotient (~12 fp64 ops per
// element instead of a soft-x87 add). The products p_j are the reference's
// doubles; their sum is carried exactly enough as a double-double (TwoSum),
// and the x87 chain's own roundings are bounded: each add rounds to 64 bits,
// |err_k| <= 2^-64 |s_k|, so |ip87 - sum p| <= 2^-64 (1 + 2^-30) sum_k |S_k|
// (ts below; the partial sums' low parts and second-order terms sit far inside
// the 2^-30). With y = sum p / denom as yh + yl and R bounding ip87 / denom's
// distance from it plus FDIV's own 64-bit rounding, double(FDIV result) == yh
// whenever [yh + yl - R, yh + yl + R] lies strictly between yh's two
// neighbouring rounding midpoints. quot() returns false (the caller takes the
// soft-x87 form) when that fails (a few % of random rows) or any quantity is
// outside the ranges the bound assumes (zero vectors, NaN/inf, 2^+-800).
struct IpAcc {
    double sh = 0.0, sl = 0.0, ts = 0.0, mx = 0.0;
    __device__ inline void add(double p) {
        const double s = __dadd_rn(sh, p);
        const double bb = __dsub_rn(s, sh);
        const double e = __dadd_rn(__dsub_rn(sh, __dsub_rn(s, bb)), __dsub_rn(p, bb));   // TwoSum: sh + p = s + e
        sh = s;
        sl = __dadd_rn(sl, e);
        ts = __dadd_rn(ts, fabs(s));
        mx = fmax(mx, fabs(s));
    }
    // double(ip87 / (long double)denom): 0 = certified (q exact), 1 = not
    // certified but |q - double(ip87 / denom)| <= qrad, 2 = declined (a quantity
    // outside the ranges the bound assumes; q meaningless)
    // exact: the caller certified that the x87 chain never rounded (ip_never_rounds):
    // then ip87 == sh + sl exactly and only the quotient's own roundings remain in R
    __device__ inline int quot_status(double denom, double& q, double& qrad, bool exact = false) const {
        if (!(denom >= 0x1p-800 && denom < 0x1p800 && mx >= 0x1p-800 && mx < 0x1p800 && ts < 0x1p800)) return 2;
        const double yh0 = sh / denom;
        const double r = fma(-yh0, denom, sh);             // exact remainder
        const double yl0 = __dadd_rn(r, sl) / denom;       // <= 2^-52 |yl0| off
        // renormalised: yh = the double nearest yh0 + yl0, yl its exact rest
        // (Fast2Sum, |yl0| << |yh0|). sl carries the partial sums' lost bits,
        // often several ulps of the final sum: without this step the candidate
        // yh0 is off by an ulp for ~3/4 of random rows and the check declines them.
        const double yh = __dadd_rn(yh0, yl0);
        const double yl = __dsub_rn(yl0, __dsub_rn(yh, yh0));
        const double ay = fabs(yh);
        if (!(ay >= 0x1p-800 && ay < 0x1p800)) return 2;
        const double R = ((exact ? 0.0 : __dadd_rn(ts * (0x1p-64 * (1.0 + 0x1p-30)), mx * 0x1p-88) / denom) +
                          fabs(yl0) * 0x1p-51 + ay * 0x1p-63) * (1.0 + 0x1p-20);
        const long long bits = __double_as_longlong(ay);
        const double up = __dsub_rn(__longlong_as_double(bits + 1), ay);   // ulp above |yh|
        const double dn = __dsub_rn(ay, __longlong_as_double(bits - 1));   // ulp below (half at a power of 2)
        const double dl = yh < 0.0 ? -yl : yl;
        q = yh;
        qrad = 0.0;
        if (!(__dadd_rn(dl, R) < 0.5 * up && __dsub_rn(dl, R) > -0.5 * dn)) {
            qrad = (R + fabs(yl) + 4.0 * up) * (1.0 + 0x1p-20);   // + the final double rounding
            return 1;
        }
        return 0;
    }
    __device__ inline bool quot(double denom, double& q) const {
        double qr;
        return quot_status(denom, q, qr) == 0;
    }
};

// Exponent of the lowest set bit of a nonzero value (LOWBIT_NONE for zero); for
// subnormals one below (the implicit bit counted): a lower bound, which is all
// ip_never_rounds needs.
constexpr int LOWBIT_NONE = 1 << 20;
__device__ inline int lowbit_exp(float x) {
    const uint32_t b = __float_as_uint(x);
    const int e = (int)((b >> 23) & 0xffu);
    return (b & 0x7fffffffu) == 0u ? LOWBIT_NONE : e - 150 + (int)__builtin_ctz(b | 0x800000u);
}
__device__ inline int lowbit_exp(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const int e = (int)((b >> 52) & 0x7ffu);
    return (b << 1) == 0ull ? LOWBIT_NONE : e - 1075 + (int)__builtin_ctzll(b | (1ull << 52));
}
// The x87 chain of IpAcc's products never rounded: every product p_j is a
// multiple of 2^qlow (qlow = lowbit(x) + lowbit(u) bounds lowbit(RN(x_j u_j))
// from below: a product rounds onto a grid no finer than its factors' joint
// one), and every exact partial sum S_k lies below 2^T (|S_k| <= mx (1 +
// 2^-40): mx is the largest double partial sum, off the exact one by the
// double-double rest) -- so each S_k has at most T - qlow <= 64 significant
// bits and every FADD of the chain is exact. The double-double then carries
// the same exact sums: the TwoSum rests are multiples of 2^qlow below
// 2^(T - 53), and their running sum needs at most T - 46 - qlow <= 18 bits.
__device__ inline bool ip_never_rounds(double mx, int qlow) {
    if (qlow >= LOWBIT_NONE) return true;                 // an all-zero row: every product 0
    if (!(mx > 0.0)) return mx == 0.0;
    if (!(mx < 0x1p1000)) return false;
    const int T = ilogb(mx * (1.0 + 0x1p-40)) + 1;
    return T - qlow <= 64;
}

// Cosine distance with its certificate status (IpAcc::quot_status): 0 = v is
// the reference's value, 1 = the reference's value lies within v +- rad,
// 2 = unknown. xa / cb: the row's / centroid's sequential sum of squares when
// the caller has it (row_sumsq, the prep's nbv), else < 0: formed here.
template <typename T, typename U>
__device__ inline int cosine_interval(const T* __restrict__ x, const U* __restrict__ c, int d, double& v, double& rad,
                                      double xa = -1.0, double cb = -1.0) {
    IpAcc ip;
    double a = 0.0, b = 0.0;
    const bool fa = xa < 0.0, fb = cb < 0.0;
    for (int j = 0; j < d; j++) {
        const double xj = (double)x[j], cj = (double)c[j];
        ip.add(__dmul_rn(xj, cj));
        if (fa) a = __dadd_rn(a, sq_of<T>(xj));
        if (fb) b = __dadd_rn(b, sq_of<U>(cj));
    }
    if (!fa) a = xa;
    if (!fb) b = cb;
    double q = 0.0, qr = 0.0;
    const int st = ip.quot_status(__dmul_rn(sqrt(a), sqrt(b)), q, qr);
    v = __dsub_rn(1.0, q);
    rad = st == 1 ? qr + 0x1p-50 : 0.0;      // + both roundings of 1 - q (|1 - q| < 4)
    return st;
}

template <typename T, typename U>
__device__ inline bool cosine_fast(const T* __restrict__ x, const U* __restrict__ c, int d, double& out) {
    IpAcc ip;
    double a = 0.0, b = 0.0;
    for (int j = 0; j < d; j++) {
        const double xj = (double)x[j], cj = (double)c[j];
        ip.add(__dmul_rn(xj, cj));
        a = __dadd_rn(a, sq_of<T>(xj));
        b = __dadd_rn(b, sq_of<U>(cj));
    }
    double q;
    if (!ip.quot(__dmul_rn(sqrt(a), sqrt(b)), q)) return false;
    out = __dsub_rn(1.0, q);
    return true;
}

// The same with the centroid's sequential sum of squares given (nbv, computed
// once per centroid in the reference's order).
template <typename T, typename U>
__device__ inline bool cosine_fast_nb(const T* __restrict__ x, const U* __restrict__ c, int d, double nbv, double& out) {
    IpAcc ip;
    double a = 0.0;
    for (int j = 0; j < d; j++) {
        const double xj = (double)x[j];
        ip.add(__dmul_rn(xj, (double)c[j]));
        a = __dadd_rn(a, sq_of<T>(xj));
    }
    double q;
    if (!ip.quot(__dmul_rn(sqrt(a), sqrt(nbv)), q)) return false;
    out = __dsub_rn(1.0, q);
    return true;
}

// Paths where lanes evaluate different pairs take the soft form directly: a
// wave pays the soft chain if any one lane's certificate fails (~14% of random
// pairs, mostly near-orthogonal ones), so fast + fallback inline is slower.
// The Lloyd winner path (assign.hip) lists its failures for a lane-per-row pass.
template <typename T, typename U>
__device__ inline double exact_cosine(const T* __restrict__ x, const U* __restrict__ c, int d) {
    return exact_cosine_x87(x, c, d);
}

// Either metric, `this` = x of any real type (fp32 dataset rows, fp64
// centroids), `in` = c; metric 0 = euclidean, 1 = cosine.
template <typename T, typename U>
__device__ inline double exact_dist(const T* __restrict__ x, const U* __restrict__ c, int d, int metric) {
    if (metric == 0) {
        double acc = 0.0;
        for (int j = 0; j < d; j++) {
            const double df = __dsub_rn((double)x[j], (double)c[j]);
            acc = __dadd_rn(acc, gp_sq(df));
        }
        return sqrt(acc);
    }
    return exact_cosine(x, c, d);
}

// Four consecutive row values (16-B aligned) widened to double.
__device__ inline void ld4d(const float* p, double (&o)[4]) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
__device__ inline void ld4d(const double* p, double (&o)[4]) {
    const double2 a = *reinterpret_cast<const double2*>(p), b = *reinterpret_cast<const double2*>(p + 2);
    o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
}

// x86 SSE produces one NaN from non-NaN operands: the default NaN, sign set
// (0xFFF8...), which every later operation propagates. Device NaNs are mapped
// to it wherever a reference double that may be NaN is written.
__device__ inline double x86_nan(double v) {
    return v != v ? __longlong_as_double((long long)0xFFF8000000000000ull) : v;
}
