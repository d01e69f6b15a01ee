// kmeanspp.hip — k-means++ seeding (k_means_pp, lib/clustering_phases/
// initialization.hpp:71-156) on gfx950, bit-exact with the reference.
//
// Per new centroid i = 1..K-1 the reference
//   (1) takes every row's min distance to centroids 0..i-1 (strict '<' after
//       the -1 sentinel, :88-110; its ID-keyed cache only memoises),
//   (2) the max of those minima (strict '>' from 0, :112-113),
//   (3) overwrites them with (min/max)^2 and prefix-sums them in row order,
//       in fp64 (:118-125),
//   (4) draws uniform_real<double>(0, total) and binary-searches (:127-149).
// (1) is incremental here: one exact distance per row per centroid
// (kpp_dist_kernel), the running minimum kept in HBM. (4) needs only the
// engine's canonical draws, which do not depend on the data, so the host draws
// them all up front and the whole seeding runs on the stream with no host
// round trip.
//
// (3) is a strictly sequential fp64 chain s_m = RN(s_{m-1} + q_m) over N rows.
// It is reproduced exactly, in parallel, from one observation: while s stays
// in one binade [2^e, 2^(e+1)) every s is a multiple of u = 2^(e-52), so
// RN(s + q) = s + u * RN_u(q) unless q is a tie (q/u = k + 1/2) — the chain is
// an integer prefix sum there. Rows are cut into chunks of KPP_CHUNK:
//   kpp_scan_kernel         the max of the minima; approximate chunk sums (the
//                           distance pass's sum m^2 per 256 rows / max^2) and
//                           their exclusive scan: approximate chunk starts
//   kpp_chunk_units_kernel  guess each chunk's binade from its approximate
//                           start; R = sum of RN_u(q) in units of u, or
//                           "dirty" (tie, non-finite, tiny start); chunks
//                           predicted to cross a binade, or holding a tie,
//                           also get prefix arrays in binades e and e + 1
//   kpp_chain_kernel        one wave walks the chunks with the EXACT running
//                           s: a chunk whose guess is right (s in binade e and
//                           s/u + R < 2^53) advances s by R*u exactly, 512
//                           chunks per wave-wide integer scan; a crossing or
//                           tie chunk is resolved from its prefix arrays with
//                           one hardware add per crossing / tie row; the rest
//                           (the first chunk, unresolvable rows) by hardware
//                           fp64 adds row by row. Then the draw and the
//                           reference's binary search, the prefix sums formed
//                           only for the chunk the draw lands in.
#include <climits>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "kernels.h"
#include "exact.h"

namespace lshkm {

constexpr int KPP_THREADS = 256;
constexpr int KPP_CHUNK = 512;                 // rows per chunk = 2 per thread
constexpr int KPP_DIRTY = INT_MIN;
constexpr int64_t KPP_TWO53 = 1ll << 53;

// q_m = (min_m / max)^2, as :121-124 (two roundings).
__device__ inline double kpp_q(double m, double mx) {
    const double t = __ddiv_rn(m, mx);
    return __dmul_rn(t, t);
}

__device__ inline double kpp_max(const unsigned long long* mx_bits) {
    return __longlong_as_double((long long)*mx_bits);
}

// Wave-level helpers of the exact walk (one wave, every lane active): an
// inclusive int64 scan by DPP row shifts inside each 16-lane row plus the row
// totals by readlane (no LDS round trips, unlike __shfl_up), and reads of a
// uniform lane.
__device__ inline int64_t dpp_shr64(int64_t v, int k) {
    const int lo = (int)(uint32_t)(uint64_t)v, hi = (int)(uint32_t)((uint64_t)v >> 32);
    int rl, rh;
    switch (k) {   // row_shr:k (0x110 + k); lanes without a source read 0 (bound_ctrl)
        case 1: rl = __builtin_amdgcn_update_dpp(0, lo, 0x111, 0xF, 0xF, true); rh = __builtin_amdgcn_update_dpp(0, hi, 0x111, 0xF, 0xF, true); break;
        case 2: rl = __builtin_amdgcn_update_dpp(0, lo, 0x112, 0xF, 0xF, true); rh = __builtin_amdgcn_update_dpp(0, hi, 0x112, 0xF, 0xF, true); break;
        case 4: rl = __builtin_amdgcn_update_dpp(0, lo, 0x114, 0xF, 0xF, true); rh = __builtin_amdgcn_update_dpp(0, hi, 0x114, 0xF, 0xF, true); break;
        default: rl = __builtin_amdgcn_update_dpp(0, lo, 0x118, 0xF, 0xF, true); rh = __builtin_amdgcn_update_dpp(0, hi, 0x118, 0xF, 0xF, true); break;
    }
    return (int64_t)(((uint64_t)(uint32_t)rh << 32) | (uint32_t)rl);
}
__device__ inline int64_t readlane64(int64_t v, int l) {
    const int lo = __builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, l);
    const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ inline int64_t wave_incl_scan64(int64_t v, int lane) {
    v += dpp_shr64(v, 1);
    v += dpp_shr64(v, 2);
    v += dpp_shr64(v, 4);
    v += dpp_shr64(v, 8);
    const int64_t t0 = readlane64(v, 15), t1 = readlane64(v, 31), t2 = readlane64(v, 47);
    const int row = lane >> 4;
    return v + (row > 0 ? t0 : 0) + (row > 1 ? t1 : 0) + (row > 2 ? t2 : 0);
}

// Binade exponent of a positive normal double (s in [2^e, 2^(e+1))).
__device__ inline int kpp_binade(double s) {
    return (int)((__double_as_longlong(s) >> 52) & 0x7ff) - 1023;
}

// ------------------------------------------------------------- (1) + (2)
// Distances of every row to the newest centroid (row chosen[it-1]), the
// running minimum, and the max of the minima (positive doubles order as their
// bit patterns; the reference's max starts at 0 with '>', so only m > 0 count).
// A block owns 256 rows (one per thread) and streams them through LDS in
// slices of KPP_DJ dims, loaded coalesced (consecutive lanes, consecutive
// floats of a row); each thread then accumulates its row in dim order, exactly
// as exact.h. The centroid row is read with uniform (scalar) loads.
// VEC (d % 32 == 0): each slice is 8 float4 per thread, all in flight at
// once, and the next slice's loads are issued before the current one is
// consumed (register double buffer).
constexpr int KPP_DJ = 32;
constexpr int KPP_V4 = KPP_THREADS * KPP_DJ / 4 / KPP_THREADS;   // float4 per thread per slice (8)

// The max of the minima: each block writes its own (positive doubles order as
// their bit patterns; 0 when it has none) and kpp_max_reduce_kernel folds them
// -- one global atomic per wave on a single word serialised at ~12 ns each
// (15,600 waves at N = 1M: ~0.19 ms of the 0.25 ms distance pass).
__device__ inline void kpp_block_max(double best, unsigned long long* __restrict__ bmax) {
    __shared__ double wbest[KPP_THREADS / 64];
    for (int off = 32; off >= 1; off >>= 1) {
        const double o = __shfl_xor(best, off);
        if (o > best) best = o;
    }
    if ((threadIdx.x & 63) == 0) wbest[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = 0.0;
        for (int w = 0; w < KPP_THREADS / 64; w++)
            if (wbest[w] > b) b = wbest[w];
        bmax[blockIdx.x] = (unsigned long long)__double_as_longlong(b);
    }
}

// Sum of the block's m^2 (any order: only the chunk guesses use it) for its
// 256-row group g. Every thread of the block calls it.
__device__ inline void kpp_group_sum(double v, double* __restrict__ gsum, int64_t g) {
    __shared__ double wsum[KPP_THREADS / 64];
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < KPP_THREADS / 64; w++) t += wsum[w];
        gsum[g] = t;
    }
    __syncthreads();
}

// TX: fp32 or fp64 rows (VEC only for fp32).
template <int METRIC, bool VEC, typename TX>
__global__ __launch_bounds__(KPP_THREADS) void kpp_dist_kernel(const TX* __restrict__ X, int64_t N, int d,
                                                               const int32_t* __restrict__ chosen, int it,
                                                               double* __restrict__ mind,
                                                               unsigned long long* __restrict__ bmax,
                                                               double* __restrict__ gsum) {
    static_assert(!VEC || sizeof(TX) == 4, "the float4 form reads fp32 rows");
    constexpr int DJ = sizeof(TX) == 4 ? KPP_DJ : KPP_DJ / 2;     // tile <= 34 KiB either way
    __shared__ TX tile[KPP_THREADS][DJ + 1];
    __shared__ double sqs[METRIC == 0 ? KPP_THREADS / 64 : 1][64 * 8];   // gp_sq_wave: 64 * 8 per wave
    double* sqb = sqs[METRIC == 0 ? threadIdx.x >> 6 : 0];
    // the newest centroid's row, widened to fp64 once per block (LDS broadcast
    // reads in the chain instead of a uniform global load per dim)
    extern __shared__ __attribute__((aligned(8))) char kpp_dyn[];
    TX* cs = reinterpret_cast<TX*>(kpp_dyn);            // [d] (dynamic)
    const TX* __restrict__ c = X + (int64_t)chosen[it - 1] * d;
    for (int j = threadIdx.x; j < d; j += KPP_THREADS) cs[j] = c[j];
    __syncthreads();
    double cb = 0.0;                                    // cosine: sum c^2 (uniform)
    if (METRIC == 1)
        for (int j = 0; j < d; j++) {
            const double cj = (double)cs[j];
            cb = __dadd_rn(cb, sq_of<TX>(cj));
        }
    double best = 0.0;
    for (int64_t row0 = (int64_t)blockIdx.x * KPP_THREADS; row0 < N; row0 += (int64_t)gridDim.x * KPP_THREADS) {
        const int64_t n = row0 + threadIdx.x;
        const int rows = (int)(N - row0 < KPP_THREADS ? N - row0 : KPP_THREADS);
        double acc = 0.0, a = 0.0;
        X87acc ip;
        ip.init();
        float4 pf[KPP_V4];
        if (VEC) {
#pragma unroll
            for (int k = 0; k < KPP_V4; k++) {
                const int idx = k * KPP_THREADS + threadIdx.x, r = idx >> 3, part = idx & 7;
                if (r < rows) pf[k] = *reinterpret_cast<const float4*>(X + (row0 + r) * d + part * 4);
            }
        }
        for (int j0 = 0; j0 < d; j0 += DJ) {
            const int dj = d - j0 < DJ ? d - j0 : DJ;
            __syncthreads();
            if (VEC) {
#pragma unroll
                for (int k = 0; k < KPP_V4; k++) {
                    const int idx = k * KPP_THREADS + threadIdx.x, r = idx >> 3, part = idx & 7;
                    if (r < rows) {
                        tile[r][part * 4 + 0] = pf[k].x;
                        tile[r][part * 4 + 1] = pf[k].y;
                        tile[r][part * 4 + 2] = pf[k].z;
                        tile[r][part * 4 + 3] = pf[k].w;
                    }
                }
            } else {
#pragma unroll 4
                for (int e = threadIdx.x; e < KPP_THREADS * DJ; e += KPP_THREADS) {
                    const int r = e / DJ, jj = e % DJ;
                    if (r < rows && jj < dj) tile[r][jj] = X[(row0 + r) * d + j0 + jj];
                }
            }
            __syncthreads();
            if (VEC && j0 + DJ < d) {
#pragma unroll
                for (int k = 0; k < KPP_V4; k++) {
                    const int idx = k * KPP_THREADS + threadIdx.x, r = idx >> 3, part = idx & 7;
                    if (r < rows)
                        pf[k] = *reinterpret_cast<const float4*>(X + (row0 + r) * d + j0 + DJ + part * 4);
                }
            }
            if (METRIC == 0) {
                // the whole block (rows past N too: their sums are dropped), the
                // squares through gp_sq_wave (glibc's pow batched over the wave)
                int jj = 0;
#pragma unroll 1
                for (; jj + 8 <= dj; jj += 8) {
                    double df[8], p[8];
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        df[q] = __dsub_rn((double)tile[threadIdx.x][jj + q], (double)cs[j0 + jj + q]);
                    gp_sq_wave<8, sizeof(TX) == 8>(df, p, sqb);
#pragma unroll
                    for (int q = 0; q < 8; q++) acc = __dadd_rn(acc, p[q]);
                }
#pragma unroll 1
                for (; jj < dj; jj++) {
                    const double df[1] = {__dsub_rn((double)tile[threadIdx.x][jj], (double)cs[j0 + jj])};
                    double p[1];
                    gp_sq_wave<1, sizeof(TX) == 8>(df, p, sqb);
                    acc = __dadd_rn(acc, p[0]);
                }
            } else if (n < N) {
#pragma unroll 8
                for (int jj = 0; jj < dj; jj++) {
                    const double xj = (double)tile[threadIdx.x][jj];
                    const double cj = (double)cs[j0 + jj];
                    ip.add(__dmul_rn(xj, cj));
                    a = __dadd_rn(a, sq_of<TX>(xj));
                }
            }
        }
        double m = 0.0;
        if (n < N) {
        double dd;
        if (METRIC == 0) {
            dd = sqrt(acc);
        } else {
            const double denom = __dmul_rn(sqrt(a), sqrt(cb));
            dd = one_minus(x87_quot(ip.value(), denom));
        }
        m = dd;
        if (it > 1) {
            const double prev = mind[n];
            if (!(dd < prev)) m = prev;
        }
        mind[n] = m;
        if (m > best) best = m;
        }
        kpp_group_sum(m * m, gsum, row0 / KPP_THREADS);
    }
    kpp_block_max(best, bmax);
}

// Euclidean on fp32 rows with d % 32 == 0 (16-B aligned rows): each wave takes
// 64 consecutive rows and reads them 16 dims at a time as 16-B pieces, four
// lanes per row's 64 contiguous bytes (a row per lane touched 64 lines per
// load instruction), transposed through LDS with the next step's loads in
// flight; the squares go through gp_sq_wave (glibc's pow batched over the
// wave). The centroid row is an LDS broadcast. Same exact-order chain as above.
constexpr int KR_S = 20;                                 // LDS row stride of the transpose (floats)
__global__ __launch_bounds__(KPP_THREADS) void kpp_dist_reg_kernel(const float* __restrict__ X, int64_t N, int d,
                                                                   const int32_t* __restrict__ chosen, int it,
                                                                   double* __restrict__ mind,
                                                                   unsigned long long* __restrict__ bmax,
                                                                   double* __restrict__ gsum) {
    extern __shared__ __attribute__((aligned(8))) char kpp_dyn2[];
    float* cs = reinterpret_cast<float*>(kpp_dyn2);     // [d]
    __shared__ double sqs[KPP_THREADS / 64][64 * 16];   // gp_sq_wave: 64 * 16 per wave
    __shared__ __attribute__((aligned(16))) float trs[KPP_THREADS / 64][64 * KR_S];
    const float* __restrict__ c = X + (int64_t)chosen[it - 1] * d;
    for (int j = threadIdx.x; j < d; j += KPP_THREADS) cs[j] = c[j];
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double* sqb = sqs[w];
    float* tr = trs[w];
    double best = 0.0;
    for (int64_t row0 = (int64_t)blockIdx.x * KPP_THREADS; row0 < N; row0 += (int64_t)gridDim.x * KPP_THREADS) {
        const int64_t wr0 = row0 + 64 * w;             // this wave's rows wr0 .. wr0 + 63 (past N: row N - 1, dropped)
        const int64_t n = wr0 + lane;
        // this lane's 4 pieces: rows wr0 + q / 4 (q = 64 k + lane), dims 4 (q % 4) of each 16-dim step
        const int64_t r0 = wr0 + (lane >> 2), rlast = N - 1;
        const float* s0 = X + (r0 < N ? r0 : rlast) * d + 4 * (lane & 3);
        const float* s1 = X + (r0 + 16 < N ? r0 + 16 : rlast) * d + 4 * (lane & 3);
        const float* s2 = X + (r0 + 32 < N ? r0 + 32 : rlast) * d + 4 * (lane & 3);
        const float* s3 = X + (r0 + 48 < N ? r0 + 48 : rlast) * d + 4 * (lane & 3);
        float* t0 = tr + (lane >> 2) * KR_S + 4 * (lane & 3);
        float4 n0 = *reinterpret_cast<const float4*>(s0), n1 = *reinterpret_cast<const float4*>(s1);
        float4 n2 = *reinterpret_cast<const float4*>(s2), n3 = *reinterpret_cast<const float4*>(s3);
        double acc = 0.0;
        for (int j0 = 0; j0 < d; j0 += 16) {
            const float4 c0 = n0, c1 = n1, c2 = n2, c3 = n3;
            const int jn = j0 + 16 < d ? j0 + 16 : j0;     // the last step reloads its own (no branch)
            n0 = *reinterpret_cast<const float4*>(s0 + jn);
            n1 = *reinterpret_cast<const float4*>(s1 + jn);
            n2 = *reinterpret_cast<const float4*>(s2 + jn);
            n3 = *reinterpret_cast<const float4*>(s3 + jn);
            *reinterpret_cast<float4*>(t0) = c0;
            *reinterpret_cast<float4*>(t0 + 16 * KR_S) = c1;
            *reinterpret_cast<float4*>(t0 + 32 * KR_S) = c2;
            *reinterpret_cast<float4*>(t0 + 48 * KR_S) = c3;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            double df[16], p[16];
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const float4 v = *reinterpret_cast<const float4*>(tr + lane * KR_S + 4 * h);
                const float xv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int u = 0; u < 4; u++) df[4 * h + u] = __dsub_rn((double)xv[u], (double)cs[j0 + 4 * h + u]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            gp_sq_wave<16, false>(df, p, sqb);
#pragma unroll
            for (int u = 0; u < 16; u++) acc = __dadd_rn(acc, p[u]);
        }
        double m = 0.0;
        if (n < N) {
            const double dd = sqrt(acc);
            m = dd;
            if (it > 1) {
                const double prev = mind[n];
                if (!(dd < prev)) m = prev;
            }
            mind[n] = m;
            if (m > best) best = m;
        }
        kpp_group_sum(m * m, gsum, row0 / KPP_THREADS);
    }
    kpp_block_max(best, bmax);
}

// --------------------------------------------------------------------- (3)
// One block: the max of the minima (from the per-block maxima, written to
// mx_bits for the exact q_m), then the approximate chunk sums sum m^2 / max^2
// (two 256-row groups per chunk) and their exclusive scan (order irrelevant:
// guesses only).
constexpr int KPP_SCAN_THREADS = 1024;
static_assert(KPP_CHUNK == 2 * KPP_THREADS, "two row groups per chunk");

__global__ __launch_bounds__(KPP_SCAN_THREADS) void kpp_scan_kernel(const unsigned long long* __restrict__ bmax, int nb,
                                                                    const double* __restrict__ gsum, int64_t ngroups,
                                                                    int64_t nch, unsigned long long* __restrict__ mx_bits,
                                                                    double* __restrict__ chunk_start) {
    __shared__ unsigned long long redm[KPP_SCAN_THREADS];
    __shared__ double part[KPP_SCAN_THREADS];
    unsigned long long mb = 0;
    for (int i = threadIdx.x; i < nb; i += KPP_SCAN_THREADS) mb = bmax[i] > mb ? bmax[i] : mb;
    redm[threadIdx.x] = mb;
    __syncthreads();
    for (int off = KPP_SCAN_THREADS / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off && redm[threadIdx.x + off] > redm[threadIdx.x]) redm[threadIdx.x] = redm[threadIdx.x + off];
        __syncthreads();
    }
    const unsigned long long mxb = redm[0];
    if (threadIdx.x == 0) *mx_bits = mxb;
    const double mx = __longlong_as_double((long long)mxb);
    const double inv = 1.0 / (mx * mx);
    auto csum = [&](int64_t c) { return (gsum[2 * c] + (2 * c + 1 < ngroups ? gsum[2 * c + 1] : 0.0)) * inv; };
    const int64_t per = (nch + KPP_SCAN_THREADS - 1) / KPP_SCAN_THREADS;
    const int64_t lo = threadIdx.x * per, hi = lo + per < nch ? lo + per : nch;
    double v = 0.0;
    for (int64_t c = lo; c < hi; c++) v += csum(c);
    part[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < KPP_SCAN_THREADS; off <<= 1) {   // inclusive scan of the partials
        const double o = (int)threadIdx.x >= off ? part[threadIdx.x - off] : 0.0;
        __syncthreads();
        part[threadIdx.x] += o;
        __syncthreads();
    }
    double run = threadIdx.x ? part[threadIdx.x - 1] : 0.0;
    for (int64_t c = lo; c < hi; c++) {
        chunk_start[c] = run;
        run += csum(c);
    }
}

// RN_u(q) in units of u = 2^(e-52), or -1 if q cannot be resolved in binade e
// (non-finite, q >= 2^(e+1), or an exact tie).
__device__ inline int64_t kpp_units(double q, int e) {
    if (!(q >= 0.0) || !(q < __longlong_as_double((long long)(e + 1 + 1023) << 52))) return -1;
    const double t = ldexp(q, 52 - e);          // exact: t < 2^53
    const double r = floor(t);
    const double f = t - r;                     // exact
    if (f == 0.5) return -1;
    return (int64_t)r + (f > 0.5 ? 1 : 0);
}

struct KppChunk {
    int64_t R;     // sum of the chunk's RN_u(q) in units of 2^(e-52)
    int32_t e;     // guessed binade, or KPP_DIRTY
    int32_t dual;  // 0, or 2048 + the guessed binade eg: prefix arrays in eg, eg + 1 in pa / pb
};
// prefix-array entries: the inclusive prefix of RN_u(q) (a tie counted as its
// floor) | KPP_TIE if the row itself is a tie; negative from an unresolvable
// row (non-finite, q >= 2^(e+1)) on. Prefixes stay below 512 * 2^53 = 2^62.
constexpr int64_t KPP_TIE = 1ll << 62;
constexpr int64_t KPP_PMASK = KPP_TIE - 1;
constexpr int64_t KPP_POISON = INT64_MIN;

// RN_u(q) in units of u = 2^(e-52) with its class: 0 resolved, 1 a tie (the
// floor returned: the rounding depends on the running sum's parity), 2 not
// resolvable in binade e (non-finite, q >= 2^(e+1); 0 returned).
__device__ inline int64_t kpp_units_c(double q, int e, int& cls) {
    if (!(q >= 0.0) || !(q < __longlong_as_double((long long)(e + 1 + 1023) << 52))) { cls = 2; return 0; }
    const double t = ldexp(q, 52 - e);
    const double r = floor(t);
    const double f = t - r;
    cls = f == 0.5 ? 1 : 0;
    return (int64_t)r + (f > 0.5 ? 1 : 0);
}

// Chunk guesses. A chunk the running sum is predicted to cross (the next
// chunk's approximate start lies in a higher binade, or its own sum leaves the
// binade) or that holds a tie also gets its prefix arrays in binades e and
// e + 1 (pa, pb), so the walk resolves it with one hardware add per crossing
// or tie row instead of element by element. Thread t owns rows 2t, 2t+1 (row
// order for the scans).
__global__ __launch_bounds__(KPP_THREADS) void kpp_chunk_units_kernel(const double* __restrict__ mind, int64_t N,
                                                                      const unsigned long long* __restrict__ mx_bits,
                                                                      double* __restrict__ qbuf,
                                                                      const double* __restrict__ chunk_start, int64_t nch,
                                                                      KppChunk* __restrict__ meta,
                                                                      int64_t* __restrict__ pa, int64_t* __restrict__ pb) {
    static_assert(KPP_CHUNK == 2 * KPP_THREADS, "two rows per thread");
    __shared__ long long red[KPP_THREADS / 64];
    __shared__ int redc[KPP_THREADS / 64];
    __shared__ long long wtot[4][KPP_THREADS / 64];
    const int64_t c0 = (int64_t)blockIdx.x * KPP_CHUNK;
    const double a = chunk_start[blockIdx.x];
    // a guess only; tiny or non-finite starts are left to the exact walk
    const bool usable = a >= 0x1p-900 && a < 0x1p62;
    const int e = usable ? kpp_binade(a) : 0;
    const int64_t i0 = c0 + 2 * threadIdx.x;
    // q_m = (min_m / max)^2 (:121-124), stored for the walk
    const double mx = kpp_max(mx_bits);
    const double q0 = i0 < N ? kpp_q(mind[i0], mx) : 0.0, q1 = i0 + 1 < N ? kpp_q(mind[i0 + 1], mx) : 0.0;
    if (i0 < N) qbuf[i0] = q0;
    if (i0 + 1 < N) qbuf[i0 + 1] = q1;
    int ca0, ca1;
    const int64_t ra0 = kpp_units_c(q0, e, ca0), ra1 = kpp_units_c(q1, e, ca1);
    long long v = ra0 + ra1;
    int cl = ca0 | ca1;
    for (int off = 32; off >= 1; off >>= 1) {
        v += __shfl_xor(v, off);
        cl |= __shfl_xor(cl, off);
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { red[w] = v; redc[w] = cl; }
    __syncthreads();
    long long t = 0;
    int any = 0;
    for (int k = 0; k < KPP_THREADS / 64; k++) { t += red[k]; any |= redc[k]; }
    const bool cross = usable && (t >= KPP_TWO53 || (blockIdx.x + 1 < nch && !(chunk_start[blockIdx.x + 1] <
                                                                            __longlong_as_double((long long)(e + 1 + 1023) << 52))));
    const bool arrays = usable && (cross || (any & 1));
    if (arrays) {                                  // block-uniform
        int cb0, cb1;
        const int64_t rb0 = kpp_units_c(q0, e + 1, cb0), rb1 = kpp_units_c(q1, e + 1, cb1);
        // values and unresolvable-row counts, scanned in row order
        int64_t sa = wave_incl_scan64(ra0 + ra1, lane), sb = wave_incl_scan64(rb0 + rb1, lane);
        int64_t sfa = wave_incl_scan64((ca0 == 2) + (ca1 == 2), lane), sfb = wave_incl_scan64((cb0 == 2) + (cb1 == 2), lane);
        if (lane == 63) { wtot[0][w] = sa; wtot[1][w] = sb; wtot[2][w] = sfa; wtot[3][w] = sfb; }
        __syncthreads();
        for (int k = 0; k < w; k++) { sa += wtot[0][k]; sb += wtot[1][k]; sfa += wtot[2][k]; sfb += wtot[3][k]; }
        // inclusive prefixes at rows 2t and 2t + 1
        auto enc = [](int64_t p, int64_t bad, int cls) { return bad ? KPP_POISON : p | (cls == 1 ? KPP_TIE : 0); };
        if (i0 < N) {
            pa[i0] = enc(sa - ra1, sfa - (ca1 == 2), ca0);
            pb[i0] = enc(sb - rb1, sfb - (cb1 == 2), cb0);
        }
        if (i0 + 1 < N) {
            pa[i0 + 1] = enc(sa, sfa, ca1);
            pb[i0 + 1] = enc(sb, sfb, cb1);
        }
    }
    if (threadIdx.x == 0) {
        KppChunk m;
        // a tie or unresolvable row makes the chunk dirty (the walk stops
        // there); R >= 2^53 (it leaves the binade) stops it as well
        const bool dirty = !usable || any != 0;
        m.R = dirty ? 0 : t;
        m.e = dirty ? KPP_DIRTY : e;
        m.dual = arrays ? 2048 + e : 0;
        meta[blockIdx.x] = m;
    }
}

// The exact walk (one wave). s is uniform across the wave. A step covers
// 64 lanes x CPL consecutive chunks (lane-local prefix, then a wave scan of
// the lane totals); R < 2^53 per chunk keeps every prefix below 2^62.
__global__ __launch_bounds__(64) void kpp_chain_kernel(const double* __restrict__ qbuf, int64_t N,
                                                       const KppChunk* __restrict__ meta, int64_t nch,
                                                       const int64_t* __restrict__ pa, const int64_t* __restrict__ pb,
                                                       double* chunk_s, int32_t* chunk_mode,
                                                       double* cum, const double* __restrict__ canon, int it,
                                                       int32_t* __restrict__ chosen, unsigned long long* __restrict__ stats) {
    constexpr int CPL = 8;                         // chunks per lane per step
    constexpr int STEP = 64 * CPL;
    constexpr int WIN = 2 * STEP;                  // chunk metadata staged in LDS (16 KB)
    __shared__ KppChunk wm[WIN];
    __shared__ double qs[KPP_CHUNK];
    __shared__ int64_t pas[KPP_CHUNK], pbs[KPP_CHUNK];
    const int lane = threadIdx.x;
    double s = 0.0;
    int64_t base = 0, win0 = -2 * WIN;
    unsigned long long nseq = 0;
#if defined(KPP_PROF)
    unsigned long long tp[5] = {0, 0, 0, 0, 0}, npass = 0;
    unsigned long long tq = __builtin_amdgcn_s_memtime();
#define KPP_T(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); tp[i] += t_ - tq; tq = t_; }
#else
#define KPP_T(i)
#endif
    while (base < nch) {
        KPP_T(4)
        if (base < win0 || base + STEP > win0 + WIN) {   // (re)fill the window at base
            win0 = base;
            // all loads in flight before the LDS writes (clamped indices: a guarded
            // load per element compiled to one round trip each)
            KppChunk tmp[WIN / 64];
#pragma unroll
            for (int t = 0; t < WIN / 64; t++) {
                const int64_t j = win0 + lane + 64 * t;
                tmp[t] = meta[j < nch ? j : nch - 1];
            }
#pragma unroll
            for (int t = 0; t < WIN / 64; t++) wm[lane + 64 * t] = tmp[t];
            wave_sync();
        }
        KPP_T(0)
        const bool s_ok = s >= 0x1p-900 && s < 0x1p62;
        const int es = s_ok ? kpp_binade(s) : 0;
        const int64_t s_units = s_ok ? (int64_t)ldexp(s, 52 - es) : 0;
        const int64_t j0 = base + (int64_t)lane * CPL;
        int64_t R[CPL];
        int lbad = CPL;                            // first chunk of the lane with a wrong guess
        int64_t tot = 0;
#pragma unroll
        for (int t = 0; t < CPL; t++) {
            const int64_t j = j0 + t;
            KppChunk m;
            m.R = 0; m.e = KPP_DIRTY;
            if (j < nch) m = wm[j - win0];
            R[t] = m.R;
            tot += m.R;
            if (lbad == CPL && !(j < nch && s_ok && m.e == es)) lbad = t;
        }
        // exclusive prefix of the lane totals
        int64_t pre = wave_incl_scan64(tot, lane) - tot;
        // the lane's first chunk that is wrong or would leave the binade
        int first = lbad;
        int64_t run = s_units + pre;
#pragma unroll
        for (int t = 0; t < CPL; t++) {
            if (t < first && run + R[t] >= KPP_TWO53) first = t;
            if (t < first) run += R[t];
        }
        const unsigned long long bad = __ballot(first < CPL);
        const int fl = bad ? __ffsll((long long)bad) - 1 : 64;       // first lane with a stop
        // lanes before fl: all CPL chunks resolved; lane fl: its chunks before
        // `first` (lanes before fl have first == CPL)
        if (lane <= fl) {
            int64_t r = s_units + pre;
#pragma unroll
            for (int t = 0; t < CPL; t++) {
                if (t < first) {
                    chunk_s[j0 + t] = ldexp((double)r, es - 52);
                    chunk_mode[j0 + t] = 0;
                    r += R[t];
                }
            }
        }
        const int fstop = fl < 64 ? __builtin_amdgcn_readlane(first, fl) : CPL;
        const int64_t c = base + (int64_t)(fl < 64 ? fl : 64) * CPL + (fl < 64 ? fstop : 0);
        // s after the resolved chunks: `run` of lane fl (or of lane 63 if none stopped)
        const int64_t adv = readlane64(run, fl < 64 ? fl : 63);
        if (c > base) s = ldexp((double)adv, es - 52);
        if (fl == 64) {
            base += STEP;
            continue;
        }
        if (c >= nch) break;
        if (c >= win0 + WIN) {                     // not a stop, just the window's end
            base = c;
            continue;
        }
        // Stop chunk c (the first, a binade crossing, a tie, a non-finite value).
        // With prefix arrays (a predicted crossing): the rows before the crossing
        // from pa in s's binade, the crossing row by the reference's hardware add,
        // the rows after it from pb in the next binade, all in parallel. Any rest
        // (no arrays, a tie, a second crossing): the reference's adds one by one
        // (:122-125), s uniform in every lane, ~26 cycles per row.
        KPP_T(1)
        const int64_t r0 = c * KPP_CHUNK;
        const int n = (int)(N - r0 < KPP_CHUNK ? N - r0 : KPP_CHUNK);
        if (lane == 0) {
            chunk_s[c] = s;
            chunk_mode[c] = 1;
        }
        const KppChunk mc = wm[c - win0];
        const bool arrays = mc.dual != 0;
        const int eg = mc.dual - 2048;
        // lane l holds rows 8l..8l+7 of the prefix arrays in registers; q and the
        // arrays also go to LDS for the uniform reads; every load is issued
        // before the first use (clamped indices)
        constexpr int EPL = KPP_CHUNK / 64;
        int64_t PA[EPL], PB[EPL];
        {
            double qv[EPL];
#pragma unroll
            for (int t = 0; t < EPL; t++) {
                const int i = lane * EPL + t;
                qv[t] = qbuf[r0 + (i < n ? i : n - 1)];
            }
            if (arrays) {
#pragma unroll
                for (int t = 0; t < EPL; t++) {
                    const int i = lane * EPL + t;
                    PA[t] = pa[r0 + (i < n ? i : n - 1)];
                    PB[t] = pb[r0 + (i < n ? i : n - 1)];
                }
            }
#pragma unroll
            for (int t = 0; t < EPL; t++) qs[lane * EPL + t] = qv[t];
            if (arrays) {
#pragma unroll
                for (int t = 0; t < EPL; t++) { pas[lane * EPL + t] = PA[t]; pbs[lane * EPL + t] = PB[t]; }
            }
        }
        wave_sync();
        KPP_T(2)
        // rows [i0, m) resolved as integers in binade E from the prefix array P
        // (s exact, in binade E): returns m, the first row that is a tie,
        // unresolvable or leaves the binade; s advances to row m - 1
        auto resolve = [&](const int64_t* P, const int64_t (&PR)[EPL], int i0, int E) -> int {
            const int64_t su = (int64_t)ldexp(s, 52 - E);
            const int64_t base_p = i0 > 0 ? (P[i0 - 1] & KPP_PMASK) : 0;
            int lf = EPL;
#pragma unroll
            for (int t = 0; t < EPL; t++) {
                const int i = lane * EPL + t;
                const int64_t p = PR[t];
                if (lf == EPL && i >= i0 && i < n &&
                    (p < 0 || (p & KPP_TIE) || su + ((p & KPP_PMASK) - base_p) >= KPP_TWO53))
                    lf = t;
            }
            const unsigned long long fbits = __ballot(lf < EPL);
            const int fl = fbits ? __ffsll((long long)fbits) - 1 : 64;
            const int m = fl < 64 ? fl * EPL + __builtin_amdgcn_readlane(lf, fl) : n;
            double out[EPL];
#pragma unroll
            for (int t = 0; t < EPL; t++) out[t] = ldexp((double)(su + ((PR[t] & KPP_PMASK) - base_p)), E - 52);
#pragma unroll
            for (int t = 0; t < EPL; t++) {
                const int i = lane * EPL + t;
                if (i >= i0 && i < m) cum[r0 + i] = out[t];
            }
            if (m > i0) s = ldexp((double)(su + ((P[m - 1] & KPP_PMASK) - base_p)), E - 52);
            return m;
        };
        int i0 = 0;
        while (arrays && i0 < n) {
            if (!(s >= 0x1p-900 && s < 0x1p62)) break;
            const int E = kpp_binade(s);
            if (E != eg && E != eg + 1) break;
            const int64_t* P = E == eg ? pas : pbs;
            i0 = E == eg ? resolve(pas, PA, i0, E) : resolve(pbs, PB, i0, E);
            if (i0 >= n || P[i0] < 0) break;         // done, or an unresolvable row: one by one from it
            s = __dadd_rn(qs[i0], s);               // a tie or crossing row: the reference's add
            if (lane == 0) cum[r0 + i0] = s;
            i0++;
        }
#if defined(KPP_PROF)
        npass += n - i0;
#if defined(KPP_PROF_STOPS)
        if (lane == 0) printf("KPPSTOP %lld %d %d %d %d %d\n", (long long)c, mc.dual, mc.e, es, (int)s_ok, i0);
#endif
#endif
        // the rest one by one: every lane adds and stores the same value (one
        // line, no exec toggling), the next 16 values read ahead from LDS with
        // uniform-address (broadcast) reads
        constexpr int QB = 16;
        double qn[QB];
#pragma unroll
        for (int t = 0; t < QB; t++) qn[t] = qs[i0 + t < n ? i0 + t : n - 1];
        int i = i0;
        for (; i + QB <= n; i += QB) {
            double qv[QB];
#pragma unroll
            for (int t = 0; t < QB; t++) qv[t] = qn[t];
            if (i + 2 * QB <= n) {
#pragma unroll
                for (int t = 0; t < QB; t++) qn[t] = qs[i + QB + t];
            }
#pragma unroll
            for (int t = 0; t < QB; t++) {
                s = __dadd_rn(qv[t], s);           // the reference's add (0 + q_0 = q_0 for row 0)
                cum[r0 + i + t] = s;
            }
        }
        for (; i < n; i++) {
            s = __dadd_rn(qs[i], s);
            cum[r0 + i] = s;
        }
        wave_sync();
        KPP_T(3)
        base = c + 1;
        nseq++;
    }
    // ---- (4) the draw (:127-149): rd = uniform_real(0, total) = canon * (total -
    // 0) + 0, then the reference's binary search = the first row whose prefix
    // sum reaches rd (the sums never decrease, rd <= total; a NaN total from
    // degenerate minima gives rd NaN and row 0). The prefix sums are never
    // materialised: the chunk by a 64-ary search over the chunk ends, then its
    // rows (the walk wrote a stop chunk's; an integer chunk's are formed here).
    {
        __threadfence();                           // this wave's chunk_s / cum stores, visible to its loads
        const double total = s;
        const double rd = __dadd_rn(__dmul_rn(canon[it], __dsub_rn(total, 0.0)), 0.0);
        int64_t pick = 0;
        if (rd > qbuf[0]) {                        // cum[0] = 0 + q_0 = q_0
            auto chunk_end = [&](int64_t cc) -> double { return cc + 1 < nch ? chunk_s[cc + 1] : total; };
            int64_t lo = 0, hi = nch;              // the first chunk whose end reaches rd lies in [lo, hi)
            while (hi - lo > 64) {
                const int64_t step = (hi - lo + 63) / 64;
                const int64_t p = lo + (int64_t)(lane + 1) * step - 1;
                const bool ge = p >= hi - 1 || chunk_end(p) >= rd;
                const unsigned long long b = __ballot(ge);
                const int f = __ffsll((long long)b) - 1;          // lane 63 always qualifies
                const int64_t nlo = f > 0 ? lo + (int64_t)f * step : lo;
                const int64_t nhi = lo + (int64_t)(f + 1) * step;
                lo = nlo;
                hi = nhi < hi ? nhi : hi;
            }
            const bool ge = lo + lane >= hi - 1 || chunk_end(lo + lane) >= rd;
            const int64_t cs_ = lo + (__ffsll((long long)__ballot(ge)) - 1);
            // rows of chunk cs_
            const int64_t r0 = cs_ * KPP_CHUNK;
            const int n = (int)(N - r0 < KPP_CHUNK ? N - r0 : KPP_CHUNK);
            constexpr int EPL = KPP_CHUNK / 64;
            double v[EPL];
            if (chunk_mode[cs_] != 0) {
#pragma unroll
                for (int t = 0; t < EPL; t++) {
                    const int i = lane * EPL + t;
                    v[t] = cum[r0 + (i < n ? i : n - 1)];
                }
            } else {
                const int e = meta[cs_].e;
                const int64_t su = (int64_t)ldexp(chunk_s[cs_], 52 - e);
                int64_t r[EPL], own = 0;
#pragma unroll
                for (int t = 0; t < EPL; t++) {
                    const int i = lane * EPL + t;
                    r[t] = i < n ? kpp_units(qbuf[r0 + i], e) : 0;
                    own += r[t];
                }
                int64_t run = su + wave_incl_scan64(own, lane) - own;
#pragma unroll
                for (int t = 0; t < EPL; t++) {
                    run += r[t];
                    v[t] = ldexp((double)run, e - 52);
                }
            }
            int lf = EPL;
#pragma unroll
            for (int t = 0; t < EPL; t++)
                if (lf == EPL && lane * EPL + t < n && v[t] >= rd) lf = t;
            const unsigned long long b = __ballot(lf < EPL);
            const int fl = b ? __ffsll((long long)b) - 1 : 63;      // b != 0: the chunk's end reaches rd
            pick = r0 + fl * EPL + __builtin_amdgcn_readlane(lf, fl);
        }
        if (lane == 0) chosen[it] = (int32_t)pick;
    }
#if defined(KPP_PROF)
    if (lane == 0) printf("KPPPROF %llu %llu %llu %llu %llu %llu %llu\n", tp[0], tp[1], tp[2], tp[3], tp[4], nseq, npass);
#endif
    if (lane == 0 && stats) {
        atomicAdd(stats + STAT_KPP_CHUNKS, (unsigned long long)nch);
        atomicAdd(stats + STAT_KPP_SEQ, nseq);
    }
}

// Runs iterations 1..K-1; chosen[0] and canon[1..K-1] are already on the device.
// ws: mind[N] f64, cum[N] f64, then per chunk sum/start f64, meta, s_start f64,
// mode i32, and the max word.
int launch_kmeans_pp(hipStream_t s, Pts X, int64_t N, int d, int K, int metric, const double* canon,
                     int32_t* chosen, void* ws, unsigned long long* stats) {

    const int64_t nch = (N + KPP_CHUNK - 1) / KPP_CHUNK;
    char* p = (char*)ws;
    double* mind = (double*)p;                 p += sizeof(double) * N;
    double* cum = (double*)p;                  p += sizeof(double) * N;
    const int64_t ngroups = (N + KPP_THREADS - 1) / KPP_THREADS;
    double* gsum = (double*)p;                 p += sizeof(double) * ((ngroups + 1) & ~1ll);   // per 256-row group sum m^2
    double* cstart = (double*)p;               p += sizeof(double) * nch;
    KppChunk* meta = (KppChunk*)p;             p += sizeof(KppChunk) * nch;
    double* cs = (double*)p;                   p += sizeof(double) * nch;
    int32_t* mode = (int32_t*)p;               p += sizeof(int32_t) * ((nch + 1) & ~1ll);
    unsigned long long* mx = (unsigned long long*)p;   p += 64;
    unsigned long long* bmax = (unsigned long long*)p;   p += 4096 * 8;   // [<= 4096] per-block maxima
    double* qbuf = (double*)p;                 p += sizeof(double) * N;   // [N] q_m
    int64_t* pa = (int64_t*)p;                 p += sizeof(int64_t) * N;  // crossing chunks' prefix arrays
    int64_t* pb = (int64_t*)p;
    const unsigned dgrid = gsz(N, KPP_THREADS, 4096);
    for (int it = 1; it < K; it++) {

        const bool vec = d % KPP_DJ == 0 && !X.f64;
        const dim3 g(dgrid), b(KPP_THREADS);
        const size_t ld32 = (size_t)d * 4, ld64 = (size_t)d * 8;     // the centroid row in LDS
        if (X.f64) {
            if (metric == 0) hipLaunchKernelGGL((kpp_dist_kernel<0, false, double>), g, b, ld64, s, X.d(), N, d, chosen, it, mind, bmax, gsum);
            else hipLaunchKernelGGL((kpp_dist_kernel<1, false, double>), g, b, ld64, s, X.d(), N, d, chosen, it, mind, bmax, gsum);
        } else if (metric == 0 && vec)
            hipLaunchKernelGGL(kpp_dist_reg_kernel, g, b, ld32, s, X.f(), N, d, chosen, it, mind, bmax, gsum);
        else if (metric == 0)
            hipLaunchKernelGGL((kpp_dist_kernel<0, false, float>), g, b, ld32, s, X.f(), N, d, chosen, it, mind, bmax, gsum);
        else if (vec)
            hipLaunchKernelGGL((kpp_dist_kernel<1, true, float>), g, b, ld32, s, X.f(), N, d, chosen, it, mind, bmax, gsum);
        else
            hipLaunchKernelGGL((kpp_dist_kernel<1, false, float>), g, b, ld32, s, X.f(), N, d, chosen, it, mind, bmax, gsum);
        hipLaunchKernelGGL(kpp_scan_kernel, dim3(1), dim3(KPP_SCAN_THREADS), 0, s, bmax, (int)dgrid, gsum, ngroups, nch, mx, cstart);
        hipLaunchKernelGGL(kpp_chunk_units_kernel, dim3((unsigned)nch), dim3(KPP_THREADS), 0, s, mind, N, mx, qbuf, cstart, nch, meta,
                           pa, pb);
        hipLaunchKernelGGL(kpp_chain_kernel, dim3(1), dim3(64), 0, s, qbuf, N, meta, nch, pa, pb, cs, mode, cum, canon, it,
                           chosen, stats);
        const int rc = kstatus("kmeanspp.hip");
        if (rc) return rc;
    }
    return 0;
}

size_t kmeans_pp_ws_bytes(int64_t N) {
    const int64_t nch = (N + KPP_CHUNK - 1) / KPP_CHUNK;
    const int64_t ngroups = (N + KPP_THREADS - 1) / KPP_THREADS;
    return sizeof(double) * 2 * (size_t)N + sizeof(double) * (size_t)((ngroups + 1) & ~1ll) +
           (sizeof(double) * 2 + sizeof(KppChunk)) * (size_t)nch +
           sizeof(int32_t) * (size_t)((nch + 1) & ~1ll) + 64 + 4096 * 8 + sizeof(double) * (size_t)N +
           2 * sizeof(int64_t) * (size_t)N;
}

}  // namespace lshkm
