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
#include "common.h"
#include "kernels.h"
#include "exact.h"

namespace lshkm {

constexpr int KM_U = 16;

__global__ __launch_bounds__(64) void km_chain_kernel(const float* __restrict__ X, int d, const int32_t* __restrict__ rows,
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
    double s = carry ? carry[(size_t)c * d + j] : 0.0;
    int64_t p = beg;
    for (; p + KM_U <= end; p += KM_U) {
        float v[KM_U];
#pragma unroll
        for (int u = 0; u < KM_U; u++) v[u] = X[(int64_t)r4[p + u] * d + j];
#pragma unroll
        for (int u = 0; u < KM_U; u++) s = __dadd_rn(s, (double)v[u]);
    }
    for (; p < end; p++) s = __dadd_rn(s, (double)X[(int64_t)r4[p] * d + j]);
    sums[(size_t)c * d + j] = s;
}

int launch_km_chain(hipStream_t s, const float* X, int d, const int32_t* rows, const int64_t* crow, int K,
                    double* sums, int64_t* counts, const double* carry, const int64_t* carry_counts) {
    hipLaunchKernelGGL(km_chain_kernel, dim3((unsigned)K, (unsigned)((d + 63) / 64)), dim3(64), 0, s, X, d, rows, crow, K,
                       carry, carry_counts, sums, counts);
    return kstatus("update.hip");
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
            acc = __dadd_rn(acc, __dmul_rn(df, df));
        }
        dist = sqrt(acc);
    } else {
        sx80 ip = sx_zero();
        double x = 0.0, y = 0.0;
        for (int j = 0; j < d; j++) {
            ip = sx_add_double(ip, __dmul_rn(a[j], b[j]));
            x = __dadd_rn(x, __dmul_rn(a[j], a[j]));
            y = __dadd_rn(y, __dmul_rn(b[j], b[j]));
        }
        const double denom = __dmul_rn(sqrt(x), sqrt(y));
        dist = one_minus(x87_quot(ip, denom));
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
