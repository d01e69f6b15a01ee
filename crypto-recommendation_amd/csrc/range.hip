// range.hip — LSH / hypercube range assignment on gfx950.
//
// Replaces:
//   lsh_range_assignment / cube_range_assignment  lib/clustering_phases/assignment.hpp:108-145
//   range_assignment                              assignment.hpp:148-217
//   lloyds_for_remaining                          assignment.hpp:83-104 (via the Lloyd path)
//   find_min_vector_distance                      lib/utils.hpp:161-178
//
// The reference walks centroid i's combined bucket for i = 0..K-1 and doubles
// the radius after every centroid, repeating whole passes until one assigns
// nothing. Everything a step reads or writes belongs to one row (its cluster,
// its distance, its distanceMap entries keyed "<centroid id>to<row id>"), and
// the radii are fixed by the step index alone: step s = pass*K + i runs with
// radius r0 * 2^s and min_radius r0 * 2^(s-1) (0 at s = 0) — repeated doubling
// is exact up to overflow, like ldexp. So each row replays, in order, only the
// steps whose bucket holds it: the (row, centroid) incidences of the combined
// buckets sorted by row (stable, so centroids stay ascending), one thread per
// row, one launch per pass; the pass count decides termination exactly as
// `assigned_count` does.
//
// The distance cache matters only when two centroids share an ID (every
// "k_means_center" after k_means, update.hpp:46): key[i] groups them, and the
// first distance computed for (group, row) is the one every later lookup sees.
#include "common.h"
#include "exact.h"
#include "kernels.h"

namespace lshkm {

// find_min_vector_distance over the centroid rows, /2: the sequential scan
// with the -1 sentinel keeps the first pair's value if it is NaN and is
// otherwise the minimum of the non-NaN values (the sign of a zero never
// reaches a comparison downstream).
// Many blocks, one pair per thread iteration (a single block ran K^2 / 1024
// sequential exact chains per thread: 2.4 ms at K = 256); the minimum is an
// atomicMin over order-preserving keys of the doubles (NaNs never enter it),
// tmp[0] = key, tmp[1] = "pair (0, 1) is NaN", tmp[2] = that NaN's bits.
constexpr int RG_MIN_THREADS = 256;
__device__ inline unsigned long long rg_key(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ inline double rg_unkey(unsigned long long k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k));
}
__global__ void rg_min_init_kernel(unsigned long long* __restrict__ tmp) {
    tmp[0] = ~0ull;
    tmp[1] = 0ull;
}
__global__ __launch_bounds__(RG_MIN_THREADS) void rg_min_pair_kernel(const double* __restrict__ C, int K, int d,
                                                                     int metric, unsigned long long* __restrict__ tmp) {
    __shared__ unsigned long long red[RG_MIN_THREADS];
    unsigned long long mk = ~0ull;
    const int64_t kk = (int64_t)K * K;
    for (int64_t p = (int64_t)blockIdx.x * RG_MIN_THREADS + threadIdx.x; p < kk; p += (int64_t)gridDim.x * RG_MIN_THREADS) {
        const int i = (int)(p / K), j = (int)(p % K);
        if (j <= i) continue;                                    // pairs (i, j > i), utils.hpp:164-165
        const double dd = exact_dist(C + (size_t)i * d, C + (size_t)j * d, d, metric);
        if (p == 1 && dd != dd) { tmp[2] = (unsigned long long)__double_as_longlong(dd); tmp[1] = 1ull; }
        if (dd == dd) mk = min(mk, rg_key(dd));
    }
    red[threadIdx.x] = mk;
    __syncthreads();
    for (int off = RG_MIN_THREADS / 2; off > 0; off >>= 1) {
        if (threadIdx.x < off) red[threadIdx.x] = min(red[threadIdx.x], red[threadIdx.x + off]);
        __syncthreads();
    }
    if (threadIdx.x == 0 && red[0] != ~0ull) atomicMin(tmp, red[0]);
}
// r0 = (first pair NaN) ? NaN / 2 : (no pairs ? -1 : min) / 2 (the reference's
// scan: a NaN first value stays, later NaNs never win a '<')
__global__ void rg_min_final_kernel(const unsigned long long* __restrict__ tmp, int K, double* __restrict__ r0) {
    const int64_t pairs = (int64_t)K * (K - 1) / 2;
    if (tmp[1]) *r0 = __longlong_as_double((long long)tmp[2]) / 2;
    else *r0 = (pairs == 0 ? -1.0 : (tmp[0] == ~0ull ? __builtin_inf() : rg_unkey(tmp[0]))) / 2;
}

// (row, centroid) incidences of the combined buckets, centroid-major.
__global__ void rg_pairs_kernel(const int64_t* __restrict__ comb_ptr, const int32_t* __restrict__ comb_idx, int K,
                                int32_t* __restrict__ rows, int32_t* __restrict__ cents) {
    for (int i = blockIdx.x; i < K; i += gridDim.x)
        for (int64_t e = comb_ptr[i] + threadIdx.x; e < comb_ptr[i + 1]; e += blockDim.x) {
            rows[e] = comb_idx[e];
            cents[e] = i;
        }
}

__global__ void rg_init_kernel(int64_t N, int32_t* __restrict__ assign, double* __restrict__ dist) {
    for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < N; n += (int64_t)gridDim.x * blockDim.x) {
        assign[n] = -1;     // remove_clustering -> resetCluster (cust_vector.hpp:205-208)
        dist[n] = 0.0;
    }
}

// One pass of the do-while loop (assignment.hpp:160-216) for every row.
// Incidence e of row n: centroid cents[e]; cache[e] / cached[e] hold the
// distanceMap entry of (key[cents[e]], n) once it exists.
template <typename TX>
__global__ void rg_pass_kernel(const TX* __restrict__ X, int d, const double* __restrict__ C, int K, int metric,
                               const int32_t* __restrict__ key, const int64_t* __restrict__ vptr,
                               const int32_t* __restrict__ cents, double* __restrict__ cache,
                               int8_t* __restrict__ cached, int64_t N, const double* __restrict__ r0p, int64_t pass,
                               int32_t* __restrict__ assign, double* __restrict__ dist,
                               unsigned long long* __restrict__ count) {
    const double r0 = *r0p;
    unsigned long long mine = 0;
    for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < N; n += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e0 = vptr[n], e1 = vptr[n + 1];
        if (e0 == e1) continue;
        int c = assign[n];
        double dc = dist[n];
        for (int64_t e = e0; e < e1; e++) {
            const int i = cents[e];
            const int64_t s = pass * K + i;
            const int sc = (int)min<int64_t>(s, 4096);          // r0 * 2^4096 has overflowed for every r0 != 0
            const double radius = ldexp(r0, sc);
            const double min_radius = s == 0 ? 0.0 : ldexp(r0, sc - 1);
            if (c == -1 || dc >= min_radius) {
                double dd;
                if (cached[e]) {
                    dd = cache[e];
                } else {
                    dd = exact_dist(X + (size_t)n * d, C + (size_t)i * d, d, metric);
                    const int g = key ? key[i] : i;
                    for (int64_t f = e0; f < e1; f++)
                        if (f == e || (key ? key[cents[f]] == g : cents[f] == i)) {
                            if (!cached[f]) { cache[f] = dd; cached[f] = 1; }
                        }
                }
                if (dd >= min_radius && dd < radius) {
                    if (c == -1 || dc > dd) { c = i; dc = dd; mine++; }
                }
            }
        }
        assign[n] = c;
        dist[n] = dc;
    }
    // the caller only tests the count for zero: a wave that assigned rows sets
    // it unless it is already set (a read instead of one serialised atomic on a
    // single word per wave, ~12 ns each)
    for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor(mine, off);
    if ((threadIdx.x & 63) == 0 && mine && __atomic_load_n(count, __ATOMIC_RELAXED) == 0ull) atomicAdd(count, mine);
}

// Rows left at -1 -> a compact list (any order: the rows are independent).
__global__ void rg_unassigned_kernel(const int32_t* __restrict__ assign, int64_t N, int32_t* __restrict__ list,
                                     unsigned long long* __restrict__ count) {
    for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < N; n += (int64_t)gridDim.x * blockDim.x) {
        const bool un = assign[n] == -1;
        const unsigned long long m = __ballot(un);
        if (!m) continue;
        const int lane = threadIdx.x & 63;
        const int leader = __builtin_ctzll(m);
        unsigned long long base = 0;
        if (lane == leader) base = atomicAdd(count, (unsigned long long)__popcll(m));
        base = __shfl(base, leader);
        if (un) list[base + __popcll(m & ((1ull << lane) - 1ull))] = (int32_t)n;
    }
}

template <typename TX>
__global__ void rg_gather_kernel(const TX* __restrict__ X, int d, const int32_t* __restrict__ list, int64_t M,
                                 TX* __restrict__ Xr) {
    const int64_t tot = M * d;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / d;
        Xr[e] = X[(size_t)list[r] * d + (e - r * d)];
    }
}

__global__ void rg_scatter_kernel(const int32_t* __restrict__ list, int64_t M, const int32_t* __restrict__ ar,
                                  const double* __restrict__ dr, int32_t* __restrict__ assign,
                                  double* __restrict__ dist) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < M; r += (int64_t)gridDim.x * blockDim.x) {
        assign[list[r]] = ar[r];
        dist[list[r]] = dr[r];
    }
}

int launch_range_radius(hipStream_t s, const double* C, int K, int d, int metric, double* r0,
                        unsigned long long* tmp) {
    const int64_t kk = (int64_t)K * K;
    hipLaunchKernelGGL(rg_min_init_kernel, dim3(1), dim3(1), 0, s, tmp);
    hipLaunchKernelGGL(rg_min_pair_kernel, dim3(gsz(kk, RG_MIN_THREADS, 2048)), dim3(RG_MIN_THREADS), 0, s, C, K, d,
                       metric, tmp);
    hipLaunchKernelGGL(rg_min_final_kernel, dim3(1), dim3(1), 0, s, tmp, K, r0);
    return kstatus("rg_min_pair_kernel");
}

int launch_range_pairs(hipStream_t s, const int64_t* comb_ptr, const int32_t* comb_idx, int K, int32_t* rows,
                       int32_t* cents) {
    hipLaunchKernelGGL(rg_pairs_kernel, dim3((unsigned)std::min(K, 4096)), dim3(256), 0, s, comb_ptr, comb_idx, K,
                       rows, cents);
    return kstatus("rg_pairs_kernel");
}

int launch_range_init(hipStream_t s, int64_t N, int32_t* assign, double* dist) {
    if (N == 0) return 0;
    hipLaunchKernelGGL(rg_init_kernel, dim3(gsz(N, 256, 8192)), dim3(256), 0, s, N, assign, dist);
    return kstatus("rg_init_kernel");
}

int launch_range_pass(hipStream_t s, Pts X, int d, const double* C, int K, int metric, const int32_t* key,
                      const int64_t* vptr, const int32_t* cents, double* cache, int8_t* cached, int64_t N,
                      const double* r0, int64_t pass, int32_t* assign, double* dist, unsigned long long* count) {
    if (N == 0) return 0;
    if (X.f64)
        hipLaunchKernelGGL(rg_pass_kernel<double>, dim3(gsz(N, 256, 16384)), dim3(256), 0, s, X.d(), d, C, K, metric,
                           key, vptr, cents, cache, cached, N, r0, pass, assign, dist, count);
    else
        hipLaunchKernelGGL(rg_pass_kernel<float>, dim3(gsz(N, 256, 16384)), dim3(256), 0, s, X.f(), d, C, K, metric,
                           key, vptr, cents, cache, cached, N, r0, pass, assign, dist, count);
    return kstatus("rg_pass_kernel");
}

int launch_range_unassigned(hipStream_t s, const int32_t* assign, int64_t N, int32_t* list,
                            unsigned long long* count) {
    if (N == 0) return 0;
    hipLaunchKernelGGL(rg_unassigned_kernel, dim3(gsz(N, 256, 8192)), dim3(256), 0, s, assign, N, list, count);
    return kstatus("rg_unassigned_kernel");
}

int launch_range_gather(hipStream_t s, Pts X, int d, const int32_t* list, int64_t M, void* Xr) {
    if (M == 0) return 0;
    if (X.f64)
        hipLaunchKernelGGL(rg_gather_kernel<double>, dim3(gsz(M * d, 256, 16384)), dim3(256), 0, s, X.d(), d, list, M,
                           static_cast<double*>(Xr));
    else
        hipLaunchKernelGGL(rg_gather_kernel<float>, dim3(gsz(M * d, 256, 16384)), dim3(256), 0, s, X.f(), d, list, M,
                           static_cast<float*>(Xr));
    return kstatus("rg_gather_kernel");
}

int launch_range_scatter(hipStream_t s, const int32_t* list, int64_t M, const int32_t* ar, const double* dr,
                         int32_t* assign, double* dist) {
    if (M == 0) return 0;
    hipLaunchKernelGGL(rg_scatter_kernel, dim3(gsz(M, 256, 8192)), dim3(256), 0, s, list, M, ar, dr, assign, dist);
    return kstatus("rg_scatter_kernel");
}

}  // namespace lshkm
