// exact.h — the reference's point-to-centroid distances in its exact
// operation order, for the device paths that need the value itself.
//   euclideanDistance  lib/data_structures/cust_vector.hpp:124-136
//     sqrt(sum_j pow(x_j - c_j, 2)), fp64, j ascending
//   cosineDistance     lib/data_structures/cust_vector.hpp:139-155
//     1 - (long double) inner product / (sqrt(sum x^2) * sqrt(sum c^2))
// `this` is the point x (fp32 values), `in` the centroid c (fp64). pow(v, 2)
// is v*v here (identical whenever v is a difference of fp32
// values, i.e. for every dataset-row centroid). No FMA contraction.
#pragma once
#include "softx87.h"

__device__ inline double exact_euclid(const float* __restrict__ x, const double* __restrict__ c, int d) {
    double acc = 0.0;
    for (int j = 0; j < d; j++) {
        const double df = __dsub_rn((double)x[j], c[j]);
        acc = __dadd_rn(acc, __dmul_rn(df, df));
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

__device__ inline double exact_cosine(const float* __restrict__ x, const double* __restrict__ c, int d) {
    sx80 ip = sx_zero();
    double a = 0.0, b = 0.0;
    for (int j = 0; j < d; j++) {
        const double xj = (double)x[j];
        ip = sx_add_double(ip, __dmul_rn(xj, c[j]));
        a = __dadd_rn(a, __dmul_rn(xj, xj));
        b = __dadd_rn(b, __dmul_rn(c[j], c[j]));
    }
    const double denom = __dmul_rn(sqrt(a), sqrt(b));
    return one_minus(x87_quot(ip, denom));
}

// Either metric, `this` = x of any real type (fp32 dataset rows, fp64
// centroids), `in` = c; metric 0 = euclidean, 1 = cosine.
template <typename T, typename U>
__device__ inline double exact_dist(const T* __restrict__ x, const U* __restrict__ c, int d, int metric) {
    if (metric == 0) {
        double acc = 0.0;
        for (int j = 0; j < d; j++) {
            const double df = __dsub_rn((double)x[j], (double)c[j]);
            acc = __dadd_rn(acc, __dmul_rn(df, df));
        }
        return sqrt(acc);
    }
    sx80 ip = sx_zero();
    double a = 0.0, b = 0.0;
    for (int j = 0; j < d; j++) {
        const double xj = (double)x[j], cj = (double)c[j];
        ip = sx_add_double(ip, __dmul_rn(xj, cj));
        a = __dadd_rn(a, __dmul_rn(xj, xj));
        b = __dadd_rn(b, __dmul_rn(cj, cj));
    }
    return one_minus(x87_quot(ip, __dmul_rn(sqrt(a), sqrt(b))));
}

// x86 SSE produces one NaN from non-NaN operands: the default NaN, sign set
// (0xFFF8...), which every later operation propagates. Device NaNs are mapped
// to it wherever a reference double that may be NaN is written.
__device__ inline double x86_nan(double v) {
    return v != v ? __longlong_as_double((long long)0xFFF8000000000000ull) : v;
}
