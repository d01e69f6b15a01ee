// update.hip — k-means center update in exact reference order on gfx950.
//
// Replaces k_means (lib/clustering_phases/update.hpp:37-86):
//   new[c][j] = ((0 + x_{i1,j}) + x_{i2,j}) + ... over the members of c in row
//   order (the `for (auto in_vector : input_vectors)` loop, :52-56, with
//   addVectorToThis, cust_vector.hpp:177-184), then / (double)count unless the
//   cluster is empty (divDimensionsByD skips 0, cust_vector.hpp:187-194);
//   continue iff some center moved more than min_dist (:63-80).
// fp64 addition is not associative, so each (c, j) is one sequential chain.
// The members of every cluster come from the stable radix sort (scatter.hip)
// in row order; a wave owns 64 dimensions of one cluster, each lane one chain,
// and streams the member rows with 16 row loads in flight per lane (row
// indices are wave-uniform scalar loads). Bytes: 4d per row read once.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "kernels.h"
#include "exact.h"
#include "kmseg.h"

namespace lshkm {

constexpr int KM_U = 16;

// One (c, j) chain over the member rows p in [beg, end), row order: groups of
// KM_U rows, loads issued three groups (48 rows) ahead of the adds so a lane
// keeps ~48 row loads in flight (the chains of large clusters were latency
// bound at 16: the k-means update of 1M fp64 rows, d = 100, K = 256 spent 5 ms
// in the longest chain). Row indices are wave-uniform (scalar loads); positions
// past the end re-read the last row and are not added.
template <typename TX>
__device__ __attribute__((always_inline)) inline double km_chain_rows(const TX* __restrict__ X, int d, int j,
                                       const __attribute__((address_space(4))) int32_t* r4, int64_t beg, int64_t end,
                                       double s) {
    if (end <= beg) return s;
    const int64_t ng = (end - beg + KM_U - 1) / KM_U;
    TX v0[KM_U], v1[KM_U], v2[KM_U], v3[KM_U];
    auto ld = [&](TX (&v)[KM_U], int64_t g) {
        const int64_t p0 = beg + g * KM_U;
        if (p0 + KM_U <= end) {          // 16 contiguous indices: one scalar block load
            const auto* rp = r4 + p0;
#pragma unroll
            for (int u = 0; u < KM_U; u++) v[u] = X[(int64_t)rp[u] * d + j];
        } else {
#pragma unroll
            for (int u = 0; u < KM_U; u++) v[u] = X[(int64_t)r4[min(p0 + u, end - 1)] * d + j];
        }
    };
    auto add = [&](const TX (&v)[KM_U], int64_t g) {
        const int64_t p0 = beg + g * KM_U;
        if (p0 + KM_U <= end) {
#pragma unroll
            for (int u = 0; u < KM_U; u++) s = __dadd_rn(s, (double)v[u]);
        } else {
#pragma unroll
            for (int u = 0; u < KM_U; u++)
                if (p0 + u < end) s = __dadd_rn(s, (double)v[u]);
        }
    };
    ld(v0, 0);
    ld(v1, 1);
    ld(v2, 2);
    for (int64_t g = 0; g < ng; g += 4) {
        ld(v3, g + 3);
        add(v0, g);
        if (g + 1 >= ng) break;
        ld(v0, g + 4);
        add(v1, g + 1);
        if (g + 2 >= ng) break;
        ld(v1, g + 5);
        add(v2, g + 2);
        if (g + 3 >= ng) break;
        ld(v2, g + 6);
        add(v3, g + 3);
    }
    return s;
}

// Wide form (the sequential chains of large clusters): a wave owns 16 dims of
// one cluster and each load instruction fetches 4 member rows (lane group k =
// lane >> 4 the row, lane & 15 the dim), so a wave keeps 4 x 48 rows in flight
// and the d / 16 waves of a cluster run side by side (the 64-dim form held one
// row per instruction and two waves per cluster at d = 100; the largest
// cluster's chain set the time). The chain lanes (k = 0) take the other groups'
// values by lane-half swaps, in row order. Member indices are read one group of
// 64 ahead of the row loads that use them.
constexpr int KM16_G = 64;                 // member positions per group (16 steps x 4 rows)
constexpr int KM16_Q = 3;                  // groups of row loads in flight

__device__ inline double km_x16(double v) {      // lanes k = 0, 2: lane + 16's value
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_permlane16_swap((uint32_t)b, (uint32_t)b, false, false)[1];
    const uint32_t hi = __builtin_amdgcn_permlane16_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false)[1];
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ inline double km_x32(double v) {      // lanes k = 0, 1: lane + 32's value
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false)[1];
    const uint32_t hi = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false)[1];
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

template <typename TX>
__global__ __launch_bounds__(64) void km_chain16_kernel(const TX* __restrict__ X, int d, const int32_t* __restrict__ rows,
                                                       const int64_t* __restrict__ crow, const double* __restrict__ carry,
                                                       const int* __restrict__ flag, double* __restrict__ sums,
                                                       const uint8_t* __restrict__ mask) {
    const int c = blockIdx.x, jb = blockIdx.y;
    if (flag && !((flag[c] >> min(31, jb / 4)) & 1)) return;
    const int lane = threadIdx.x, k = lane >> 4;
    const int j = jb * 16 + (lane & 15);
    const int jl = j < d ? j : d - 1;
    const int64_t beg = crow[c], end = crow[c + 1];
    double s = carry && j < d ? carry[(size_t)c * d + j] : 0.0;
    const int64_t ng = (end - beg + KM16_G - 1) / KM16_G;
    auto idx = [&](int64_t gi) {
        const int64_t p = beg + gi * KM16_G + lane;
        return rows[p < end ? p : (end > beg ? end - 1 : beg)];
    };
    TX v[KM16_Q + 1][16];
    auto ld = [&](TX (&vv)[16], int32_t ri) {
#pragma unroll
        for (int st = 0; st < 16; st++) {
            const int rr = __shfl(ri, 4 * st + k);
            vv[st] = X[(int64_t)rr * d + jl];
        }
    };
    auto add = [&](const TX (&vv)[16], int64_t gi) {
        const int64_t p0 = beg + gi * KM16_G;
        const bool full = p0 + KM16_G <= end;
#pragma unroll
        for (int st = 0; st < 16; st++) {
            const double x0 = (double)vv[st];
            const double x1 = km_x16(x0), x2 = km_x32(x0), x3 = km_x32(km_x16(x0));
            const int64_t p = p0 + 4 * st;
            if (full) {
                s = __dadd_rn(s, x0); s = __dadd_rn(s, x1); s = __dadd_rn(s, x2); s = __dadd_rn(s, x3);
            } else {
                if (p < end) s = __dadd_rn(s, x0);
                if (p + 1 < end) s = __dadd_rn(s, x1);
                if (p + 2 < end) s = __dadd_rn(s, x2);
                if (p + 3 < end) s = __dadd_rn(s, x3);
            }
        }
    };
    if (ng > 0) {
        // indices one group ahead of the loads that use them
        int32_t r_next = idx(0);
        int32_t r_after = idx(1);
#pragma unroll
        for (int q = 0; q < KM16_Q; q++) {
            ld(v[q], r_next);
            r_next = r_after;
            r_after = idx(q + 2);
        }
        for (int64_t g = 0; g < ng; g += KM16_Q + 1) {
#pragma unroll
            for (int u = 0; u <= KM16_Q; u++) {
                if (g + u >= ng) break;
                ld(v[(u + KM16_Q) % (KM16_Q + 1)], r_next);     // group g + u + Q (past the end: re-reads)
                r_next = r_after;
                r_after = idx(g + u + KM16_Q + 2);
                add(v[u], g + u);
            }
        }
    }
    if (k == 0 && j < d && (!mask || mask[(size_t)c * d + j])) sums[(size_t)c * d + j] = s;
}

template <typename TX>
__global__ __launch_bounds__(64) void km_chain_kernel(const TX* __restrict__ X, int d, const int32_t* __restrict__ rows,
                                                     const int64_t* __restrict__ crow, int K,
                                                     const double* __restrict__ carry, const int64_t* __restrict__ carry_counts,
                                                     double* __restrict__ sums, int64_t* __restrict__ counts) {
    const int c = blockIdx.x;
    const int j = blockIdx.y * 64 + threadIdx.x;
    const int64_t beg = crow[c], end = crow[c + 1];
    if (blockIdx.y == 0 && threadIdx.x == 0 && counts) counts[c] = end - beg + (carry_counts ? carry_counts[c] : 0);
    if (j >= d) return;
    const __attribute__((address_space(4))) int32_t* r4 = (const __attribute__((address_space(4))) int32_t*)rows;
    // exact mode across shards: the chain continues from the previous shard's running sum
    const double s = km_chain_rows(X, d, j, r4, beg, end, carry ? carry[(size_t)c * d + j] : 0.0);
    sums[(size_t)c * d + j] = s;
}

__global__ void km_counts_kernel(const int64_t* __restrict__ crow, int K, const int64_t* __restrict__ carry_counts,
                                 int64_t* __restrict__ counts) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < K) counts[c] = crow[c + 1] - crow[c] + (carry_counts ? carry_counts[c] : 0);
}

static bool km_wide() {
    // the wide form (16 dims per wave, 4 member rows per load) by default: the
    // fp64 update of 1M x 100 rows, K = 256, 3.44 -> 2.68 ms; LSHKM_KM_CHAIN=64:
    // the 64-dim form
    return !test_switch("LSHKM_KM_CHAIN", "64");
}

int launch_km_chain(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K,
                    double* sums, int64_t* counts, const double* carry, const int64_t* carry_counts) {
    if (km_wide()) {
        const dim3 grid((unsigned)K, (unsigned)((d + 15) / 16));
        if (X.f64)
            hipLaunchKernelGGL(km_chain16_kernel<double>, grid, dim3(64), 0, s, X.d(), d, rows, crow, carry, nullptr, sums, nullptr);
        else
            hipLaunchKernelGGL(km_chain16_kernel<float>, grid, dim3(64), 0, s, X.f(), d, rows, crow, carry, nullptr, sums, nullptr);
        if (counts)
            hipLaunchKernelGGL(km_counts_kernel, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, s, crow, K, carry_counts,
                               counts);
        return kstatus("update.hip");
    }
    const dim3 grid((unsigned)K, (unsigned)((d + 63) / 64));
    if (X.f64)
        hipLaunchKernelGGL(km_chain_kernel<double>, grid, dim3(64), 0, s, X.d(), d, rows, crow, K, carry, carry_counts,
                           sums, counts);
    else
        hipLaunchKernelGGL(km_chain_kernel<float>, grid, dim3(64), 0, s, X.f(), d, rows, crow, K, carry, carry_counts,
                           sums, counts);
    return kstatus("update.hip");
}

// ------------------------------------------------------------------ parallel form
// The reference's chain s = ((0 + x_1) + x_2) + ... rounds only when a partial
// sum is not a double. Every partial sum -- of the chain, or of any subset of
// the values in any order -- is an integer multiple of 2^q (q = the lowest set
// bit over the chain's values) bounded by A = sum |x_i| < count * 2^t (t = the
// highest bit position + 1), so when ceil(log2 count) + t - q <= 53 every such
// partial is a double: no step of the chain rounds, and neither does any other
// order of fp64 additions. The chain's result is then the exact sum, which
// plain fp64 adds compute in any order -- per lane, then by fp64 atomics into
// the (c, j) accumulator. q and t are tracked alongside (integer min / max), and
// a chain whose test fails (or holding inf / nan) is flagged and recomputed by
// the sequential kernel above (km_chain_kernel).
// Work: waves stream 512 consecutive member positions of the cluster-sorted
// list (lane = dimension), flushing their partial (one fp64 atomic add, two
// integer atomics) whenever the cluster changes.
constexpr int KMF_CH = 512;
constexpr int KMF_BAD = 1 << 20;     // qmin marker of a chain that needs the sequential kernel

struct KmFx {                        // per (c, j), zeroed / initialised by km_fx_init_kernel
    double sum;
    double asum;                     // sum of |x| (rounded: <= (1 + n 2^-53) times the true one)
    int qmin;                        // lowest set-bit exponent, -KMF_BAD if flagged
    int tmax;                        // highest bit position + 1
};

__global__ void km_fx_init_kernel(KmFx* __restrict__ acc, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { acc[i].sum = 0.0; acc[i].asum = 0.0; acc[i].qmin = 1 << 30; acc[i].tmax = -(1 << 30); }
}

__device__ inline void km_fx_flush(KmFx* a, double v, double av, int qmin, int tmax, bool bad) {
    if (v != 0.0) atomicAdd(&a->sum, v);
    if (av != 0.0) atomicAdd(&a->asum, av);
    atomicMin(&a->qmin, bad ? -KMF_BAD : qmin);
    atomicMax(&a->tmax, tmax);
}

// The never-rounds test of one (c, j): its cnt values are integer multiples of
// 2^qmin below 2^tmax in magnitude, and their |x| sum to asum (fp64-rounded in
// any order: within a factor 1 + cnt 2^-53 <= 1 + 2^-22 of the true sum for
// cnt < 2^31). Every partial sum of any subset, in any order, is a multiple of
// 2^qmin no larger in magnitude than the true sum of |x|: a double when that is
// below 2^(53 + qmin). The count form (cnt 2^tmax) is the coarser bound of the
// same kind; the |x| form passes on far more general fp32 chains (N(0,1) rows:
// ~95 % vs ~64 % of the chains of 10K values).
__device__ inline bool km_cert(int qmin, int tmax, int64_t cnt, double asum) {
    if (qmin <= -KMF_BAD / 2) return false;        // inf / nan among the values
    if (qmin > tmax) return true;                  // no nonzero value: the sum is +0
    int lc = 0;
    while (((int64_t)1 << lc) < cnt) lc++;         // ceil(log2 count)
    // every partial below cnt 2^tmax <= 2^(lc + tmax): finite only if that is <=
    // 2^1023 (else an any-order sum may overflow where the reference's chain stays
    // finite, e.g. [M, -M, M] with M = 1.5 * 2^1023)
    if (lc + tmax - qmin <= 53 && lc + tmax <= 1023) return true;
    // the |x| bound (an overflowed asum is inf and fails; 2^(53 + qmin) may be inf)
    return asum * (1.0 + 0x1p-20) < ldexp(1.0, min(53 + qmin, 1024));
}

// lowest set-bit exponent q and top t of a nonzero finite value; false for
// +-0 (adds nothing: -0 + 0 = +0 either way) and inf / nan (sets bad)
__device__ inline bool km_fx_bits(float v, int& q, int& t, bool& bad) {
    const uint32_t b = __float_as_uint(v);
    const int E = (int)((b >> 23) & 255u);
    const uint32_t f = b & 0x7FFFFFu;
    if (E == 255) { bad = true; return false; }
    const uint32_t m = E ? (f | 0x800000u) : f;
    if (m == 0) return false;
    const int e = (E ? E : 1) - 150;
    q = e + __builtin_ctz(m);
    t = e + 32 - __builtin_clz(m);
    return true;
}
__device__ inline bool km_fx_bits(double v, int& q, int& t, bool& bad) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const int E = (int)((b >> 52) & 2047u);
    const uint64_t f = b & 0xFFFFFFFFFFFFFull;
    if (E == 2047) { bad = true; return false; }
    const uint64_t m = E ? (f | (1ull << 52)) : f;
    if (m == 0) return false;
    const int e = (E ? E : 1) - 1075;
    q = e + __builtin_ctzll(m);
    t = e + 64 - __builtin_clzll(m);
    return true;
}

template <typename TX>
__global__ __launch_bounds__(64) void km_fx_kernel(const TX* __restrict__ X, int d, const int32_t* __restrict__ rows,
                                                  const int64_t* __restrict__ crow, int K, int64_t M,
                                                  KmFx* __restrict__ acc) {
    const int64_t p0 = (int64_t)blockIdx.x * KMF_CH;
    if (p0 >= M) return;
    const int64_t p1 = min(M, p0 + KMF_CH);
    const int j = blockIdx.y * 64 + threadIdx.x;
    const bool on = j < d;
    const __attribute__((address_space(4))) int32_t* r4 = (const __attribute__((address_space(4))) int32_t*)rows;
    // cluster of position p0: the last c with crow[c] <= p0 (wave-uniform binary search)
    int lo = 0, hi = K;              // crow[lo] <= p0 < crow[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (crow[mid] <= p0) lo = mid; else hi = mid;
    }
    int c = lo;
    int64_t cend = crow[c + 1];
    double s = 0.0, as = 0.0;
    int qmin = 1 << 30, tmax = -(1 << 30);
    bool bad = false;
    for (int64_t p = p0; p < p1; p += 16) {
        TX v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = (on && p + u < p1) ? X[(int64_t)r4[p + u] * d + j] : (TX)0;
#pragma unroll
        for (int u = 0; u < 16; u++) {
            if (p + u >= p1) break;
            while (p + u >= cend) {              // cluster boundary: flush, move on (skipping empty clusters)
                if (on) km_fx_flush(acc + (size_t)c * d + j, s, as, qmin, tmax, bad);
                s = 0.0; as = 0.0; qmin = 1 << 30; tmax = -(1 << 30); bad = false;
                c++;
                cend = crow[c + 1];
            }
            int q, t;
            if (!km_fx_bits(v[u], q, t, bad)) continue;
            qmin = min(qmin, q);
            tmax = max(tmax, t);
            s = __dadd_rn(s, (double)v[u]);     // exact whenever the chain's test passes
            as = __dadd_rn(as, fabs((double)v[u]));
        }
    }
    if (on) km_fx_flush(acc + (size_t)c * d + j, s, as, qmin, tmax, bad);
}

// fp32 rows with d % 128 == 0: a wave reads whole 512-B row slices (two
// dims per lane, float2), half the load instructions of km_fx_kernel's 256-B
// half-rows for the same gather.
#ifndef KMF2_U
#define KMF2_U 16       // rows in flight per wave
#endif
__global__ __launch_bounds__(64) void km_fx2_kernel(const float* __restrict__ X, int d, const int32_t* __restrict__ rows,
                                                    const int64_t* __restrict__ crow, int K, int64_t M,
                                                    KmFx* __restrict__ acc) {
    const int64_t p0 = (int64_t)blockIdx.x * KMF_CH;
    if (p0 >= M) return;
    const int64_t p1 = min(M, p0 + KMF_CH);
    const int j = blockIdx.y * 128 + 2 * threadIdx.x;
    const __attribute__((address_space(4))) int32_t* r4 = (const __attribute__((address_space(4))) int32_t*)rows;
    int lo = 0, hi = K;              // crow[lo] <= p0 < crow[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (crow[mid] <= p0) lo = mid; else hi = mid;
    }
    int c = lo;
    int64_t cend = crow[c + 1];
    double s0 = 0.0, s1 = 0.0, a0 = 0.0, a1 = 0.0;
    int q0 = 1 << 30, t0 = -(1 << 30), q1 = 1 << 30, t1 = -(1 << 30);
    bool bad0 = false, bad1 = false;
    for (int64_t p = p0; p < p1; p += KMF2_U) {
        float2 v[KMF2_U];
#pragma unroll
        for (int u = 0; u < KMF2_U; u++)
            v[u] = p + u < p1 ? *reinterpret_cast<const float2*>(X + (int64_t)r4[p + u] * d + j) : make_float2(0.f, 0.f);
#pragma unroll
        for (int u = 0; u < KMF2_U; u++) {
            if (p + u >= p1) break;
            while (p + u >= cend) {              // cluster boundary: flush, move on (skipping empty clusters)
                km_fx_flush(acc + (size_t)c * d + j, s0, a0, q0, t0, bad0);
                km_fx_flush(acc + (size_t)c * d + j + 1, s1, a1, q1, t1, bad1);
                s0 = s1 = a0 = a1 = 0.0; q0 = q1 = 1 << 30; t0 = t1 = -(1 << 30); bad0 = bad1 = false;
                c++;
                cend = crow[c + 1];
            }
            int q, t;
            if (km_fx_bits(v[u].x, q, t, bad0)) {
                q0 = min(q0, q); t0 = max(t0, t);
                s0 = __dadd_rn(s0, (double)v[u].x);
                a0 = __dadd_rn(a0, (double)fabsf(v[u].x));
            }
            if (km_fx_bits(v[u].y, q, t, bad1)) {
                q1 = min(q1, q); t1 = max(t1, t);
                s1 = __dadd_rn(s1, (double)v[u].y);
                a1 = __dadd_rn(a1, (double)fabsf(v[u].y));
            }
        }
    }
    km_fx_flush(acc + (size_t)c * d + j, s0, a0, q0, t0, bad0);
    km_fx_flush(acc + (size_t)c * d + j + 1, s1, a1, q1, t1, bad1);
}

// The flagged chains of at most KM_LANE_MAX members (global count): one wave
// each (a lane list entry), the reference's sequential adds in member order
// from carry (NULL: 0). Lane u loads member position p0 + u of a 64-position
// block (the member indices coalesced, the values one per row), two blocks
// ahead of the adds; lane 0 adds the block's 64 values in order (readlane).
// A lane per chain left the few flagged chains of a call on a handful of CUs
// (1,016 chains: 4 blocks of 256, 7 ms); a wave per chain spreads them.
// Far cheaper than the segment passes when few chains are flagged (0.8 % of
// the C5 chains on full-mantissa rows: their 64-dim blocks touch ~40 % of the
// windows).
constexpr int64_t KM_LANE_MAX = 32768;
__device__ inline double ks_rl(double v, int i);
template <typename TX>
__global__ __launch_bounds__(64) void km_chain_lanes_kernel(const TX* __restrict__ X, int d,
                                                           const int32_t* __restrict__ rows,
                                                           const int64_t* __restrict__ crow,
                                                           const int32_t* __restrict__ list,
                                                           const unsigned int* __restrict__ count,
                                                           const double* __restrict__ carry, double* __restrict__ sums) {
    const int64_t nl = (int64_t)*count;
    const int lane = threadIdx.x;
    for (int64_t t = blockIdx.x; t < nl; t += gridDim.x) {
        const int32_t i = list[t];
        const int c = i / d, j = i - c * d;
        const int64_t beg = crow[c], end = crow[c + 1];
        double s = carry ? carry[i] : 0.0;
        auto ld = [&](int64_t p0) -> double {
            const int64_t p = min(p0 + lane, end - 1);
            return end > beg ? (double)X[(int64_t)rows[p] * d + j] : 0.0;
        };
        double v0 = ld(beg), v1 = ld(beg + 64);
        for (int64_t p0 = beg; p0 < end; p0 += 64) {
            const double v = v0;
            v0 = v1;
            v1 = ld(p0 + 128);
            const int n = (int)min((int64_t)64, end - p0);
            if (n == 64) {
#pragma unroll 16
                for (int u = 0; u < 64; u++) s = __dadd_rn(s, ks_rl(v, u));
            } else {
                for (int u = 0; u < n; u++) s = __dadd_rn(s, ks_rl(v, u));
            }
        }
        if (lane == 0) sums[i] = s;
    }
}

// Append entry i to the lane list (order kept within a wave: ballot prefix,
// one atomic per wave).
__device__ inline void km_lane_append(bool want, int32_t i, int32_t* __restrict__ list, unsigned int* __restrict__ cnt) {
    const unsigned long long m = __ballot(want);
    if (!m) return;
    const int lane = (int)(threadIdx.x & 63), leader = __builtin_ctzll(m);
    unsigned int base = 0;
    if (lane == leader) base = atomicAdd(cnt, (unsigned int)__popcll(m));
    base = __shfl(base, leader);
    if (want) list[base + __popcll(m & ((1ull << lane) - 1ull))] = i;
}

// Per (c, j): the exact sum if the chain provably never rounds, else a flag for
// the sequential kernel. carry (sharded exact mode): the chain starts from it.
__global__ void km_fx_finalize_kernel(const KmFx* __restrict__ acc, const int64_t* __restrict__ crow, int K, int d,
                                      const double* __restrict__ carry, const int64_t* __restrict__ carry_counts,
                                      double* __restrict__ sums, int* __restrict__ flag,
                                      unsigned long long* __restrict__ stat, int32_t* __restrict__ lanes,
                                      unsigned int* __restrict__ lane_cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)K * d) return;
    const int c = (int)(i / d);
    const KmFx a = acc[i];
    int64_t cnt = crow[c + 1] - crow[c];
    double s = a.sum, as = a.asum;
    int qmin = a.qmin, tmax = a.tmax;
    bool ok = qmin > -KMF_BAD / 2;
    if (carry && ok) {                  // the carried running sum is one more value of the chain
        const double s0 = carry[i];
        cnt += 1;
        int q, t;
        bool bad = false;
        if (km_fx_bits(s0, q, t, bad)) {
            qmin = min(qmin, q);
            tmax = max(tmax, t);
            s = __dadd_rn(s0, s);
            as = __dadd_rn(as, fabs(s0));
        }
        if (bad) ok = false;
    }
    ok = ok && km_cert(qmin, tmax, cnt, as);
    // a flagged chain: one lane of km_chain_lanes_kernel when it is short (and
    // a lane list is given), else its (c, 64-dim block) to the block kernels
    const bool lane_chain = !ok && lanes && cnt <= KM_LANE_MAX;
    if (ok) sums[i] = s;
    else if (!lane_chain) atomicOr(flag + c, 1 << min(31, (int)(i % d) / 64));
    if (lanes) km_lane_append(lane_chain, (int32_t)i, lanes, lane_cnt);
    if (stat) {
        const unsigned long long nb = __ballot(!ok);
        if (nb && (threadIdx.x & 63) == __builtin_ctzll(nb)) atomicAdd(stat, (unsigned long long)__popcll(nb));
    }
}

// The sequential chains of the flagged (c, 64-dim block)s only.
template <typename TX>
__global__ __launch_bounds__(64) void km_chain_flagged_kernel(const TX* __restrict__ X, int d,
                                                             const int32_t* __restrict__ rows,
                                                             const int64_t* __restrict__ crow, int K,
                                                             const double* __restrict__ carry,
                                                             const int* __restrict__ flag, double* __restrict__ sums) {
    const int c = blockIdx.x;
    if (!((flag[c] >> min(31, (int)blockIdx.y)) & 1)) return;
    const int j = blockIdx.y * 64 + threadIdx.x;
    if (j >= d) return;
    const __attribute__((address_space(4))) int32_t* r4 = (const __attribute__((address_space(4))) int32_t*)rows;
    const int64_t beg = crow[c], end = crow[c + 1];
    sums[(size_t)c * d + j] = km_chain_rows(X, d, j, r4, beg, end, carry ? carry[(size_t)c * d + j] : 0.0);
}


size_t km_fx_ws_bytes(int K, int d) { return (size_t)K * d * sizeof(KmFx) + (size_t)K * 4 + 64 + (size_t)K * d * 4 + 64; }

int launch_km_sums_seg(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                       double* sums, int64_t* counts, const double* carry, const int64_t* carry_counts, void* ws,
                       const int* flag);

int launch_km_sums_fx(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                      double* sums, int64_t* counts, const double* carry, const int64_t* carry_counts, void* ws,
                      unsigned long long* stat, void* seg_ws) {
    KmFx* acc = reinterpret_cast<KmFx*>(ws);
    int* flag = reinterpret_cast<int*>(acc + (size_t)K * d);
    unsigned int* lane_cnt = reinterpret_cast<unsigned int*>(flag + K);
    int32_t* lanes = reinterpret_cast<int32_t*>(lane_cnt + 16);
    const int64_t n = (int64_t)K * d;
    (void)hipMemsetAsync(flag, 0, (size_t)K * 4 + 64, s);      // the flags and the lane count
    hipLaunchKernelGGL(km_fx_init_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, acc, n);
    const int jb = (d + 63) / 64;
    const dim3 fgrid((unsigned)((M + KMF_CH - 1) / KMF_CH), (unsigned)jb);
    if (M > 0) {
        if (X.f64) hipLaunchKernelGGL(km_fx_kernel<double>, fgrid, dim3(64), 0, s, X.d(), d, rows, crow, K, M, acc);
        else if (d % 128 == 0)
            hipLaunchKernelGGL(km_fx2_kernel, dim3(fgrid.x, (unsigned)(d / 128)), dim3(64), 0, s, X.f(), d, rows, crow, K, M,
                               acc);
        else hipLaunchKernelGGL(km_fx_kernel<float>, fgrid, dim3(64), 0, s, X.f(), d, rows, crow, K, M, acc);
    }
    // the lane form for short flagged chains where the segment form would run
    // (test switch LSHKM_KM_LANES=0: every flagged chain to the block kernels)
    const bool use_lanes = seg_ws && !test_switch("LSHKM_KM_FLAGGED", "chain") && !test_switch("LSHKM_KM_LANES", "0");
    hipLaunchKernelGGL(km_fx_finalize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, acc, crow, K, d, carry,
                       carry_counts, sums, flag, stat, use_lanes ? lanes : nullptr, lane_cnt);
    if (use_lanes) {
        if (X.f64)
            hipLaunchKernelGGL(km_chain_lanes_kernel<double>, dim3(gsz(n, 1, 8192)), dim3(64), 0, s, X.d(), d, rows, crow,
                               lanes, lane_cnt, carry, sums);
        else
            hipLaunchKernelGGL(km_chain_lanes_kernel<float>, dim3(gsz(n, 1, 8192)), dim3(64), 0, s, X.f(), d, rows, crow,
                               lanes, lane_cnt, carry, sums);
    }
    if (seg_ws && !test_switch("LSHKM_KM_FLAGGED", "chain")) {
        // the flagged chains by binade segments (every window of theirs in
        // parallel; the sequential form's time was set by the longest chain:
        // 20 ms for a 206K-member cluster of full-mantissa rows)
        if (const int rc = launch_km_sums_seg(s, X, d, rows, crow, K, M, sums, nullptr, carry, nullptr, seg_ws, flag))
            return rc;
    } else if (km_wide()) {
        const dim3 g16((unsigned)K, (unsigned)((d + 15) / 16));
        if (X.f64)
            hipLaunchKernelGGL(km_chain16_kernel<double>, g16, dim3(64), 0, s, X.d(), d, rows, crow, carry, flag, sums, nullptr);
        else
            hipLaunchKernelGGL(km_chain16_kernel<float>, g16, dim3(64), 0, s, X.f(), d, rows, crow, carry, flag, sums, nullptr);
    } else if (X.f64)
        hipLaunchKernelGGL(km_chain_flagged_kernel<double>, dim3((unsigned)K, (unsigned)jb), dim3(64), 0, s, X.d(), d,
                           rows, crow, K, carry, flag, sums);
    else
        hipLaunchKernelGGL(km_chain_flagged_kernel<float>, dim3((unsigned)K, (unsigned)jb), dim3(64), 0, s, X.f(), d,
                           rows, crow, K, carry, flag, sums);
    if (counts)
        hipLaunchKernelGGL(km_counts_kernel, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, s, crow, K, carry_counts,
                           counts);
    return kstatus("update.hip (fixed point)");
}

// ------------------------------------------------------------------ segmented form
// fp64 rows (general doubles: the fixed-point test above fails for almost every
// chain, and the sequential chain of the largest cluster set the time). Every
// (c, j) chain is cut into pairs (512-position window x cluster) and each pair
// into binade segments (kmseg.h), four launches:
//   A ks_sum: the pair sums (any order; only to predict binades)
//   B ks_scan: the approximate sum at each pair's start, per chain
//   C ks_seg: the segment records of every pair (<= KS_R, else the pair is walked)
//   D ks_compose: one wave per chain applies the records in order (real adds
//     where a summary does not apply), so the critical path is the number of
//     segments of the longest chain, not its length.
// A and C stream the member rows (lane = dimension, 512-B row slices); pair
// (w, c) has index w + c (windows and clusters advance monotonically together).
constexpr int KS_USUM = 16;        // member rows in flight per wave: pass A
#ifndef KS_USEG
#define KS_USEG 16                 // pass C (its per-step state holds more registers)
#endif

__device__ inline int ks_first_cluster(const int64_t* __restrict__ crow, int K, int64_t p0) {
    int lo = 0, hi = K;            // crow[lo] <= p0 < crow[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (crow[mid] <= p0) lo = mid; else hi = mid;
    }
    return lo;
}

// Walk window w's positions (lane j); f(p, x) per position, close(c) when
// cluster c's part of the window ends (only for clusters with positions in it),
// open(c, p) when it starts.
template <int KS_U, typename TX, typename Open, typename Step, typename Close>
__device__ __attribute__((always_inline)) inline void ks_walk(const TX* __restrict__ X, int d, int jl,
                                                              const int32_t* __restrict__ rows,
                                                              const int64_t* __restrict__ crow, int K, int64_t M,
                                                              int64_t p0, Open&& open, Step&& step, Close&& close) {
    // positions as 32-bit offsets o = p - p0 in [0, n): scalar compares, no 64-bit VALU ones
    const int n = (int)(min(M, p0 + KS_W) - p0);
    const __attribute__((address_space(4))) int32_t* r4 =
        (const __attribute__((address_space(4))) int32_t*)rows + p0;
    int c = ks_first_cluster(crow, K, p0);
    int oend = (int)min(crow[c + 1] - p0, (int64_t)n);          // this cluster's part ends here
    open(c, p0);
    // pipeline: the member indices two blocks ahead (scalar loads), the row
    // values one block ahead; past the end, the last position again (every
    // block issues the same loads, so the waits count exactly)
    auto ld_idx = [&](int o, int32_t (&ix)[KS_U]) {
        if (o + KS_U <= n) {
#pragma unroll
            for (int u = 0; u < KS_U; u++) ix[u] = r4[o + u];
        } else {
#pragma unroll
            for (int u = 0; u < KS_U; u++) ix[u] = r4[min(o + u, n - 1)];
        }
    };
    auto ld_val = [&](const int32_t (&ix)[KS_U], double (&v)[KS_U]) {
#pragma unroll
        for (int u = 0; u < KS_U; u++) v[u] = (double)X[(int64_t)ix[u] * d + jl];
    };
    int32_t ia[KS_U], ib[KS_U];
    double va[KS_U], vb[KS_U];
    ld_idx(0, ia);
    ld_val(ia, va);
    ld_idx(KS_U, ib);
    for (int o = 0; o < n; o += KS_U) {
        ld_val(ib, vb);
        ld_idx(o + 2 * KS_U, ia);
#pragma unroll
        for (int u = 0; u < KS_U; u++) {
            if (o + u >= n) break;
            if (o + u >= oend) {                     // wave-uniform
                close(c);
                do {
                    c++;
                    oend = (int)min(crow[c + 1] - p0, (int64_t)n);
                } while (o + u >= oend);             // empty clusters have no pair here
                open(c, p0 + o + u);
            }
            step(o + u, va[u]);
        }
#pragma unroll
        for (int u = 0; u < KS_U; u++) { va[u] = vb[u]; ib[u] = ia[u]; }
    }
    close(c);
}

// flag (fp32 chains the never-rounds test flags; the sharded form): only the
// windows holding a flagged (cluster, 64-dim block) chain run; NULL: every one.
__device__ inline bool ks_window_flagged(const int* __restrict__ flag, const int64_t* __restrict__ crow, int K,
                                         int64_t M, int64_t p0) {
    if (!flag) return true;
    const int c0 = ks_first_cluster(crow, K, p0);
    const int c1 = ks_first_cluster(crow, K, min(M, p0 + KS_W) - 1);
    const int bit = min(31, (int)blockIdx.y);
    int any = 0;
    for (int c = c0; c <= c1; c++) any |= (flag[c] >> bit) & 1;
    return any != 0;
}

template <typename TX>
__global__ __launch_bounds__(64) void ks_sum_kernel(const TX* __restrict__ X, int d, const int32_t* __restrict__ rows,
                                                    const int64_t* __restrict__ crow, int K, int64_t M,
                                                    double* __restrict__ psum, const int* __restrict__ flag) {
    const int w = blockIdx.x;
    if (!ks_window_flagged(flag, crow, K, M, (int64_t)w * KS_W)) return;
    const int j = blockIdx.y * 64 + threadIdx.x;
    const bool on = j < d;
    double s = 0.0;
    ks_walk<KS_USUM>(X, d, on ? j : d - 1, rows, crow, K, M, (int64_t)w * KS_W,
            [&](int, int64_t) { s = 0.0; },
            [&](int, double x) { s += x; },
            [&](int c) { if (on) psum[(size_t)(w + c) * d + j] = s; });
}

__global__ __launch_bounds__(64) void ks_scan_kernel(const double* __restrict__ psum, const int64_t* __restrict__ crow,
                                                     int K, int d, const double* __restrict__ carry,
                                                     double* __restrict__ sin, const int* __restrict__ flag) {
    const int c = blockIdx.x;
    if (flag && !((flag[c] >> min(31, (int)blockIdx.y)) & 1)) return;
    const int j = blockIdx.y * 64 + threadIdx.x;
    const int64_t beg = crow[c], end = crow[c + 1];
    if (j >= d || beg == end) return;
    double run = carry ? carry[(size_t)c * d + j] : 0.0;
    // 16 pairs' sums loaded at once, then their (approximate) running sums: the
    // loads do not depend on the chain (a chain of 400 pairs waited on each)
    const int64_t w0 = beg / KS_W, w1 = (end - 1) / KS_W;
    for (int64_t wb = w0; wb <= w1; wb += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = wb + u <= w1 ? psum[(size_t)(wb + u + c) * d + j] : 0.0;
#pragma unroll
        for (int u = 0; u < 16; u++) {
            if (wb + u > w1) break;
            sin[(size_t)(wb + u + c) * d + j] = run;
            run += v[u];
        }
    }
}

template <typename TX>
__global__ __launch_bounds__(64) void ks_seg_kernel(const TX* __restrict__ X, int d, const int32_t* __restrict__ rows,
                                                    const int64_t* __restrict__ crow, int K, int64_t M,
                                                    const double* __restrict__ sin, int32_t* __restrict__ cnt,
                                                    KsRaw* __restrict__ rec, const int* __restrict__ flag) {
    const int w = blockIdx.x;
    if (!ks_window_flagged(flag, crow, K, M, (int64_t)w * KS_W)) return;
    const int j = blockIdx.y * 64 + threadIdx.x;
    const bool on = j < d;
    const int64_t p0 = (int64_t)w * KS_W;
    double st = 0.0;
    KsSeg g;
    bool open = false;
    int nr = 0;
    KsRaw* rp = rec;
    auto emit = [&](const KsSeg& gg) {
        if (on && nr < KS_R) rp[nr] = ks_raw(gg);
        nr++;
    };
    ks_walk<KS_USEG>(X, d, on ? j : d - 1, rows, crow, K, M, p0,
            [&](int c, int64_t) {
                const size_t o = (size_t)(w + c) * d + j;
                st = on ? sin[o] : 0.0;
                asm volatile("" : "+v"(st));      // waited here, not at every step after this branch
                open = false;
                nr = 0;
                rp = rec + o * KS_R;
            },
            [&](int o, double x) {
                st += x;
                ks_feed(g, open, x, st, o, emit);
            },
            [&](int c) {
                if (open) emit(g);
                if (on) cnt[(size_t)(w + c) * d + j] = nr;
            });
}

// D: one wave per chain. A pair's records (or, for a dense pair, its member
// values) are loaded by the lanes at once -- lane i holds record i, its bounds
// formed in every lane at once -- and applied in order by passing the running
// sum from lane to lane (DPP wave_shr:1: lane i applies record i to what lane
// i-1 produced), so the dependent chain waits on no memory load and reads no
// record through a scalar register; the next pair's count and records are in
// flight meanwhile. Each lane keeps the sum it received; one check over the
// lanes after the pass finds the first record whose summary does not apply,
// whose positions are then walked with real adds before the pass resumes.
__device__ inline double ks_rl(double v, int i) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, i);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), i);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ inline int64_t ks_rl(int64_t v, int i) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, i);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), i);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Lane form of ks_apply for the pass: every lane applies its record to its own
// sum (the result where the summary does not apply is unused).
__device__ inline double ks_apply_t(double s, const KsRec& r) {
    const double t = __dadd_rn(s, r.xa);
    const double t2 = __dadd_rn(t, r.d);
    return (t >= r.L && t <= r.H) ? t2 : t;
}
__device__ inline int ks_rec_a(uint64_t meta, int i) {
    return (int)((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)meta, i) & 0xFFFFu);
}
__device__ inline int ks_rec_b(uint64_t meta, int i) {
    return (int)(((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)meta, i) >> 16) & 0xFFFFu);
}

// Pair pipeline: while pair w is applied, pair w+1's records -- or, for a
// dense pair, its member values (lane i: positions i, i+64, ...) -- and pair
// w+2's count and member row indices are in flight (row indices always: the
// values need them one pair ahead, and a failed summary reads from them).
struct KsPair {
    int n;
    int32_t idx[KS_W / 64];
    double v[KS_W / 64];
    KsRaw r;
};
__device__ inline double ks_shr1(double v) {          // lane l <- lane l-1
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x138, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x138, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

template <typename TX>
__global__ __launch_bounds__(64) void ks_compose_kernel(const TX* __restrict__ X, int d,
                                                        const int32_t* __restrict__ rows,
                                                        const int64_t* __restrict__ crow, int K,
                                                        const double* __restrict__ carry,
                                                        const int32_t* __restrict__ cnt, const KsRaw* __restrict__ rec,
                                                        double* __restrict__ sums, const int* __restrict__ flag,
                                                        const uint8_t* __restrict__ mask) {
    const int j = blockIdx.x, c = blockIdx.y;
    const int lane = threadIdx.x;
    if (flag && !((flag[c] >> min(31, j / 64)) & 1)) return;          // the flagged chains only
    const int64_t beg = crow[c], end = crow[c + 1];
    double s = carry ? carry[(size_t)c * d + j] : 0.0;
    if (beg < end) {
        const int64_t w0 = beg / KS_W, w1 = (end - 1) / KS_W;
        auto load_meta = [&](int64_t w, KsPair& P) {      // count and row indices
            if (w > w1) return;
            P.n = cnt[(size_t)(w + c) * d + j];
            const int64_t wb = w * KS_W;
#pragma unroll
            for (int k = 0; k < KS_W / 64; k++) {
                const int64_t q = min(max(wb + 64 * k + lane, beg), end - 1);
                P.idx[k] = rows[q];
            }
        };
        auto load_body = [&](int64_t w, KsPair& P) {      // records or values
            if (w > w1) return;
            if (P.n <= KS_R) {
                if (lane < P.n) P.r = rec[((size_t)(w + c) * d + j) * KS_R + lane];
            } else {
#pragma unroll
                for (int k = 0; k < KS_W / 64; k++) P.v[k] = (double)X[(int64_t)P.idx[k] * d + j];
            }
        };
        KsPair A, B, Cn;
        load_meta(w0, A);
        load_body(w0, A);
        load_meta(w0 + 1, B);
        for (int64_t w = w0; w <= w1; w++) {
            // pair w's registers are complete before the next loads issue, so
            // nothing below waits on those (vmcnt counts in order)
            asm volatile("" : "+v"(A.r.xa), "+v"(A.r.p), "+v"(A.r.lo), "+v"(A.r.hi), "+v"(A.r.meta));
#pragma unroll
            for (int k = 0; k < KS_W / 64; k++) asm volatile("" : "+v"(A.v[k]), "+v"(A.idx[k]));
            load_meta(w + 2, Cn);
            load_body(w + 1, B);
            const int64_t wb = w * KS_W;
            const int o0 = (int)(max(beg, wb) - wb), o1 = (int)(min(end, wb + KS_W) - wb);   // valid offsets
            if (A.n > KS_R) {                            // dense pair: the plain chain
#pragma unroll
                for (int k = 0; k < KS_W / 64; k++) {
                    const int i0 = max(0, o0 - 64 * k), i1 = min(64, o1 - 64 * k);
                    if (i0 == 0 && i1 == 64) {
#pragma unroll
                        for (int i = 0; i < 64; i++) s = __dadd_rn(s, ks_rl(A.v[k], i));
                    } else {
                        for (int i = i0; i < i1; i++) s = __dadd_rn(s, ks_rl(A.v[k], i));
                    }
                }
            } else {
                const KsRec R = ks_finish(A.r);
                int i0 = 0;
                while (i0 < A.n) {
                    // records i0 .. n-1 by the pass; sin: the sum lane i received
                    double sv = s, sin = s, t = s;
                    for (int i = i0; i < A.n; i++) {
                        sin = lane == i ? sv : sin;
                        t = ks_apply_t(sv, R);
                        sv = ks_shr1(t);
                    }
                    // the first record whose summary does not apply (the lanes past it
                    // worked from a wrong sum; they are redone)
                    double ta = __dadd_rn(sin, R.xa);
                    const bool bad = lane >= i0 && lane < A.n && !(ta >= R.L && ta <= R.H);
                    const unsigned long long fb = __ballot(bad);
                    if (!fb) {
                        s = ks_rl(t, A.n - 1);
                        break;
                    }
                    const int f = __builtin_ctzll(fb);
                    s = ks_rl(ta, f);                            // the record's real first add
                    const int fa = ks_rec_a(R.meta, f), fb2 = ks_rec_b(R.meta, f);
                    // positions fa+1 .. fb2 with real adds
                    for (int k = (fa + 1) / 64; k <= fb2 / 64; k++) {
                        int32_t ix = A.idx[0];
#pragma unroll
                        for (int u = 1; u < KS_W / 64; u++) ix = u == k ? A.idx[u] : ix;   // registers, no scratch
                        const double v = (double)X[(int64_t)ix * d + j];
                        const int q0 = max(0, fa + 1 - 64 * k), q1 = min(64, fb2 + 1 - 64 * k);
                        for (int q = q0; q < q1; q++) s = __dadd_rn(s, ks_rl(v, q));
                    }
                    i0 = f + 1;
                }
            }
            A = B;
            B = Cn;
        }
    }
    if (lane == 0 && (!mask || mask[(size_t)c * d + j] == 1)) sums[(size_t)c * d + j] = s;
}

static int64_t ks_pairs(int64_t M, int K) { return (M + KS_W - 1) / KS_W + K; }

size_t km_seg_ws_bytes(int64_t M, int K, int d) {
    const size_t pd = (size_t)ks_pairs(M, K) * d;
    return pd * (8 + 8 + 4) + 64 + pd * KS_R * sizeof(KsRaw);
}

// The segment workspace: records | pair sums | pair starts | record counts.
struct KsWs {
    KsRaw* rec;
    double *psum, *sin;
    int32_t* cnt;
    KsWs(void* ws, int64_t M, int K, int d) {
        const size_t pd = (size_t)ks_pairs(M, K) * d;
        char* b = reinterpret_cast<char*>(ws);
        rec = reinterpret_cast<KsRaw*>(b);                 // 16-B aligned first
        psum = reinterpret_cast<double*>(b + pd * KS_R * sizeof(KsRaw));
        sin = psum + pd;
        cnt = reinterpret_cast<int32_t*>(sin + pd);
    }
};

// Passes A-C: the pair sums, the pairs' approximate starts (from `start`, the
// chains' approximate start values; NULL: 0) and the segment records. flag:
// only the flagged (cluster, 64-dim block) chains (NULL: all).
template <typename TX>
static void km_seg_records(hipStream_t s, const TX* X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                           const double* start, const int* flag, const KsWs& w) {
    const int jb = (d + 63) / 64;
    const int64_t W = (M + KS_W - 1) / KS_W;
    if (W <= 0) return;
    hipLaunchKernelGGL(ks_sum_kernel<TX>, dim3((unsigned)W, (unsigned)jb), dim3(64), 0, s, X, d, rows, crow, K, M, w.psum,
                       flag);
    hipLaunchKernelGGL(ks_scan_kernel, dim3((unsigned)K, (unsigned)jb), dim3(64), 0, s, w.psum, crow, K, d, start, w.sin,
                       flag);
    hipLaunchKernelGGL(ks_seg_kernel<TX>, dim3((unsigned)W, (unsigned)jb), dim3(64), 0, s, X, d, rows, crow, K, M, w.sin,
                       w.cnt, w.rec, flag);
}

// Pass D: the chains composed from `carry` (NULL: from 0); flag: only the
// flagged chains; mask: written only where set (NULL: every dim of them).
template <typename TX>
static void km_seg_compose(hipStream_t s, const TX* X, int d, const int32_t* rows, const int64_t* crow, int K,
                           const double* carry, const int* flag, const uint8_t* mask, const KsWs& w, double* sums) {
    hipLaunchKernelGGL(ks_compose_kernel<TX>, dim3((unsigned)d, (unsigned)K), dim3(64), 0, s, X, d, rows, crow, K, carry,
                       w.cnt, w.rec, sums, flag, mask);
}

// Exact-order sums by segments (sums, counts as launch_km_chain): every chain
// of fp64 rows; with flag, only the chains the never-rounds test flagged (fp32
// rows, after launch_km_sums_fx has written the others).
int launch_km_sums_seg(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                       double* sums, int64_t* counts, const double* carry, const int64_t* carry_counts, void* ws,
                       const int* flag) {
    const KsWs w(ws, M, K, d);
    if (X.f64) {
        km_seg_records(s, X.d(), d, rows, crow, K, M, carry, flag, w);
        km_seg_compose(s, X.d(), d, rows, crow, K, carry, flag, nullptr, w, sums);
    } else {
        km_seg_records(s, X.f(), d, rows, crow, K, M, carry, flag, w);
        km_seg_compose(s, X.f(), d, rows, crow, K, carry, flag, nullptr, w, sums);
    }
    if (counts)
        hipLaunchKernelGGL(km_counts_kernel, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, s, crow, K, carry_counts,
                           counts);
    return kstatus("update.hip (segmented)");
}

// ------------------------------------------------------------------ grid test
// Whether every difference of two values of X squares exactly in fp64 and
// pow(x, 2) of it is x*x (gpow2.h): all finite values are multiples of 2^q below
// 2^t with t - q <= 25 (a difference then has <= 26 significant bits) and q >=
// -460 (no square near the subnormal range). qt: [q min, t max, bad].
__global__ void grid_bits_init_kernel(int* qt) {
    qt[0] = 1 << 30;
    qt[1] = -(1 << 30);
    qt[2] = 0;
}
template <typename TX>
__global__ __launch_bounds__(256) void grid_bits_kernel(const TX* __restrict__ X, int64_t n, int* __restrict__ qt) {
    int q = 1 << 30, t = -(1 << 30);
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        int qi, ti;
        if (km_fx_bits(X[i], qi, ti, bad)) {
            q = min(q, qi);
            t = max(t, ti);
        }
    }
    // wave reductions, then one atomic per wave
    for (int o = 32; o > 0; o >>= 1) {
        q = min(q, __shfl_xor(q, o));
        t = max(t, __shfl_xor(t, o));
    }
    const bool anybad = __ballot(bad) != 0ull;
    if ((threadIdx.x & 63) == 0) {
        atomicMin(qt, q);
        atomicMax(qt + 1, t);
        if (anybad) atomicOr(qt + 2, 1);
    }
}
int launch_grid_bits(hipStream_t s, Pts X, int64_t n, int* qt) {
    hipLaunchKernelGGL(grid_bits_init_kernel, dim3(1), dim3(1), 0, s, qt);
    if (n > 0) {
        if (X.f64) hipLaunchKernelGGL(grid_bits_kernel<double>, dim3(gsz(n, 256, 4096)), dim3(256), 0, s, X.d(), n, qt);
        else hipLaunchKernelGGL(grid_bits_kernel<float>, dim3(gsz(n, 256, 4096)), dim3(256), 0, s, X.f(), n, qt);
    }
    return kstatus("update.hip (grid bits)");
}
bool grid_exact_squares(const int* qt_host) {
    return qt_host[2] == 0 && (qt_host[0] > qt_host[1] || (qt_host[1] - qt_host[0] <= 25 && qt_host[0] >= -460));
}

// ------------------------------------------------------------------ long chains
// Column sums of a row-major [n][m] fp64 block V, each column one sequential
// chain in row order from carry (NULL: 0) -- the same segmented evaluation
// with the rows as one "cluster" (iota: 0..n-1, crow: {0, n}). The clustering
// recommender's prediction chains of a huge cluster (recom.hip) take it.
__global__ void seg_iota_kernel(int32_t* __restrict__ iota, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        iota[i] = (int32_t)i;
}

size_t seg_columns_ws_bytes(int64_t n, int K, int m) { return km_seg_ws_bytes(n, K, m); }

int launch_seg_iota(hipStream_t s, int32_t* iota, int64_t n) {
    hipLaunchKernelGGL(seg_iota_kernel, dim3(gsz(n, 256, 4096)), dim3(256), 0, s, iota, n);
    return kstatus("update.hip (iota)");
}

// K blocks of rows [crow[k], crow[k+1]) of V [n][m], each column of each block
// one chain from carry[k][e] (NULL: 0) into out [K][m].
int launch_seg_columns(hipStream_t s, const double* V, int64_t n, int K, int m, const int32_t* iota,
                       const int64_t* crow, const double* carry, double* out, void* ws) {
    if (n <= 0 || m <= 0 || K <= 0) return 0;
    const KsWs w(ws, n, K, m);
    km_seg_records(s, V, m, iota, crow, K, n, carry, nullptr, w);
    km_seg_compose(s, V, m, iota, crow, K, carry, nullptr, nullptr, w, out);
    return kstatus("update.hip (column chains)");
}

// ------------------------------------------------------------------ sharded form
// The reference's chain over row shards (lshkm_kmeans_shard_*, include/lshkm.h):
// every rank forms its partial sums by the parallel form above and reports its
// values' q / t / sum |x|; after the exchange (partial sums gathered, q MIN, t
// MAX, |x| sums and counts SUM) the never-rounds test runs on the GLOBAL values.
// Where it passes, every partial sum of any subset of the chain's values, in
// any order, is a double: each rank's partial is exact, and so is the total of
// the gathered partials -- the chain's own result, whatever the order. Only the
// chains that fail it need the rank-to-rank carry, and of those only the
// composition of their segment records runs in rank order: the records are
// formed on all ranks at once from each chain's approximate start on the rank
// (the sum of the lower ranks' partials).
__global__ void km_shard_split_kernel(const KmFx* __restrict__ acc, int64_t n, double* __restrict__ sums,
                                      double* __restrict__ asum, int32_t* __restrict__ qt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const KmFx a = acc[i];
    sums[i] = a.sum;
    asum[i] = a.asum;
    qt[i] = a.qmin;
    qt[n + i] = -a.tmax;              // one MIN all-reduce for both
}

__global__ void km_shard_certify_kernel(const double* __restrict__ gathered, int world, int rank,
                                        const double* __restrict__ asum, const int32_t* __restrict__ qt,
                                        const int64_t* __restrict__ counts, int K, int d,
                                        double* __restrict__ sums_out, double* __restrict__ start,
                                        int* __restrict__ flag, uint8_t* __restrict__ mask,
                                        unsigned long long* __restrict__ nflag) {
    const int64_t n = (int64_t)K * d;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int c = (int)(i / d);
    double tot = 0.0, pre = 0.0;
    for (int r = 0; r < world; r++) {            // rank order (any order is exact where the test passes)
        if (r == rank) pre = tot;
        tot = __dadd_rn(tot, gathered[(size_t)r * n + i]);
    }
    const bool ok = km_cert(qt[i], -qt[n + i], counts[c], asum[i]);
    const bool lane_chain = !ok && counts[c] <= KM_LANE_MAX;     // the global count: the same split on every rank
    if (start) start[i] = pre;
    sums_out[i] = tot;                           // the chain's value where ok; the carry replaces the rest
    mask[i] = ok ? 0 : (lane_chain ? 2 : 1);     // 1: segment records, 2: one lane (km_chain_lanes_kernel)
    if (!ok && !lane_chain) atomicOr(flag + c, 1 << min(31, (int)(i % d) / 64));
    const unsigned long long nb = __ballot(!ok);
    if (nb && (threadIdx.x & 63) == __builtin_ctzll(nb)) atomicAdd(nflag, (unsigned long long)__popcll(nb));
}

int launch_km_shard_begin(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                          double* sums, double* asum, int32_t* qt, int64_t* counts, void* ws) {
    KmFx* acc = reinterpret_cast<KmFx*>(ws);      // the context's k-means workspace (km_fx_ws_bytes)
    const int64_t n = (int64_t)K * d;
    hipLaunchKernelGGL(km_fx_init_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, acc, n);
    const int jb = (d + 63) / 64;
    const dim3 fgrid((unsigned)((M + KMF_CH - 1) / KMF_CH), (unsigned)jb);
    if (M > 0) {
        if (X.f64) hipLaunchKernelGGL(km_fx_kernel<double>, fgrid, dim3(64), 0, s, X.d(), d, rows, crow, K, M, acc);
        else if (d % 128 == 0)
            hipLaunchKernelGGL(km_fx2_kernel, dim3(fgrid.x, (unsigned)(d / 128)), dim3(64), 0, s, X.f(), d, rows, crow, K, M,
                               acc);
        else hipLaunchKernelGGL(km_fx_kernel<float>, fgrid, dim3(64), 0, s, X.f(), d, rows, crow, K, M, acc);
    }
    hipLaunchKernelGGL(km_shard_split_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, acc, n, sums, asum, qt);
    hipLaunchKernelGGL(km_counts_kernel, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, s, crow, K, nullptr, counts);
    return kstatus("update.hip (shard begin)");
}

int launch_km_shard_certify(hipStream_t s, const double* gathered, int world, int rank, const double* asum,
                            const int32_t* qt, const int64_t* counts, int K, int d, double* sums_out, double* start,
                            int* flag, uint8_t* mask, unsigned long long* nflag) {
    const int64_t n = (int64_t)K * d;
    if (hipMemsetAsync(flag, 0, (size_t)K * 4, s) != hipSuccess || hipMemsetAsync(nflag, 0, 8, s) != hipSuccess)
        return kstatus("update.hip (shard certify memset)");
    hipLaunchKernelGGL(km_shard_certify_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, gathered, world, rank,
                       asum, qt, counts, K, d, sums_out, start, flag, mask, nflag);
    return kstatus("update.hip (shard certify)");
}

// [lane count (64 B) | lane list (K * d int32), 256-B aligned] then the
// begin pass's accumulators or the segment records
static size_t km_shard_lane_bytes(int K, int d) { return ((size_t)K * d * 4 + 64 + 255) / 256 * 256; }
size_t km_shard_ws_bytes(int64_t M, int K, int d) {
    return km_shard_lane_bytes(K, d) + std::max((size_t)K * d * sizeof(KmFx) + 64, km_seg_ws_bytes(M, K, d));
}

__global__ void km_lane_list_kernel(const uint8_t* __restrict__ mask, int64_t n, int32_t* __restrict__ list,
                                    unsigned int* __restrict__ cnt) {
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = b + threadIdx.x;
        km_lane_append(i < n && mask[i] == 2, (int32_t)i, list, cnt);
    }
}

// The flagged chains' segment records from their approximate starts on this
// rank (passes A-C, carry-free: all ranks at once).
int launch_km_shard_prepare(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                            const double* start, const int* flag, const uint8_t* mask, void* ws) {
    unsigned int* lane_cnt = reinterpret_cast<unsigned int*>(ws);
    int32_t* lanes = reinterpret_cast<int32_t*>(lane_cnt + 16);
    const int64_t n = (int64_t)K * d;
    if (hipMemsetAsync(lane_cnt, 0, 64, s) != hipSuccess) return kstatus("update.hip (shard prepare memset)");
    hipLaunchKernelGGL(km_lane_list_kernel, dim3(gsz(n, 256, 4096)), dim3(256), 0, s, mask, n, lanes, lane_cnt);
    const KsWs w(reinterpret_cast<char*>(ws) + km_shard_lane_bytes(K, d), M, K, d);
    if (X.f64) km_seg_records(s, X.d(), d, rows, crow, K, M, start, flag, w);
    else km_seg_records(s, X.f(), d, rows, crow, K, M, start, flag, w);
    return kstatus("update.hip (shard prepare)");
}

// The flagged chains composed over this rank's rows from `carry` (the previous
// rank's running sums; NULL on the first rank: from 0), written where mask is set.
int launch_km_shard_chain(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                          const int* flag, const uint8_t* mask, const double* carry, void* ws, double* sums) {
    const unsigned int* lane_cnt = reinterpret_cast<const unsigned int*>(ws);
    const int32_t* lanes = reinterpret_cast<const int32_t*>(lane_cnt + 16);
    const int64_t n = (int64_t)K * d;
    const KsWs w(reinterpret_cast<char*>(ws) + km_shard_lane_bytes(K, d), M, K, d);
    // mask 1: the segment composition (flag bits), mask 2: one lane per chain
    if (X.f64) {
        km_seg_compose(s, X.d(), d, rows, crow, K, carry, flag, mask, w, sums);
        hipLaunchKernelGGL(km_chain_lanes_kernel<double>, dim3(gsz(n, 1, 8192)), dim3(64), 0, s, X.d(), d, rows, crow,
                           lanes, lane_cnt, carry, sums);
    } else {
        km_seg_compose(s, X.f(), d, rows, crow, K, carry, flag, mask, w, sums);
        hipLaunchKernelGGL(km_chain_lanes_kernel<float>, dim3(gsz(n, 1, 8192)), dim3(64), 0, s, X.f(), d, rows, crow,
                           lanes, lane_cnt, carry, sums);
    }
    return kstatus("update.hip (shard chain)");
}

// One wave per cluster: divide (unless empty), then the reference's movement
// test with euclideanDistance(new, old) or cosineDistance(new, old).
__global__ __launch_bounds__(64) void km_finalize_kernel(const double* __restrict__ sums, const int64_t* __restrict__ counts,
                                                        int K, int d, const double* __restrict__ C_old, int metric,
                                                        double min_dist, double* __restrict__ C_new,
                                                        int* __restrict__ moved) {
    const int c = blockIdx.x;
    const double cnt = (double)counts[c];
    for (int j = threadIdx.x; j < d; j += 64) {
        const double v = sums[(size_t)c * d + j];
        C_new[(size_t)c * d + j] = cnt != 0.0 ? v / cnt : v;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    const double* a = C_new + (size_t)c * d;
    const double* b = C_old + (size_t)c * d;
    double dist;
    if (metric == 0) {
        double acc = 0.0;
        for (int j = 0; j < d; j++) {
            const double df = __dsub_rn(a[j], b[j]);
            acc = __dadd_rn(acc, gp_sq(df));
        }
        dist = sqrt(acc);
    } else {
        X87acc ip;
        ip.init();
        double x = 0.0, y = 0.0;
        for (int j = 0; j < d; j++) {
            ip.add(__dmul_rn(a[j], b[j]));
            x = __dadd_rn(x, gp_sq(a[j]));
            y = __dadd_rn(y, gp_sq(b[j]));
        }
        const double denom = __dmul_rn(sqrt(x), sqrt(y));
        dist = one_minus(x87_quot(ip.value(), denom));
    }
    if (dist > min_dist) atomicOr(moved, 1);
}

int launch_km_finalize(hipStream_t s, const double* sums, const int64_t* counts, int K, int d, const double* C_old,
                       int metric, double min_dist, double* C_new, int* moved) {
    hipLaunchKernelGGL(km_finalize_kernel, dim3((unsigned)K), dim3(64), 0, s, sums, counts, K, d, C_old, metric, min_dist,
                       C_new, moved);
    return kstatus("update.hip");
}

}  // namespace lshkm
