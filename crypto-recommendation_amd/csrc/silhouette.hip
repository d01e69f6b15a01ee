// silhouette.hip — cluster silhouettes on gfx950.
//
// Replaces: silhouette_cluster / silhouette_of_i
// (lib/clustering_phases/silhouette.hpp:31-144) over the clusters of
// separate_clusters_from_input (lib/utils.hpp:150-158).
//
//   near[c]  = argmin_{i != c} dist(centroid c, centroid i)  (-1 sentinel, strict <)
//   a(i)     = sum_{j in cluster(i)} dist(x_i, x_j)  in member order (j = i included),
//              / (|cluster| - 1) unless the cluster is a singleton
//   b(i)     = sum_{j in cluster(near[c])} dist(x_i, x_j) in member order, / |that cluster|
//   s(i)     = (b - a) / max(a, b)   (max_i = a; if (b > a) max_i = b)
//   sils[c]  = (sum of s(i) in member order) / |c|;  sils[K] = (sum over c of the
//              undivided sums, in c order) / N
// Every distance is the reference's exact one (exact.h). The reference's
// distance cache (keyed "<id>to<id>", silhouette.hpp:95-109) stores d(x_i, x_j)
// for the reverse pair; d is bitwise symmetric in both metrics (negated
// differences square alike, products and the two norms commute), so recomputing
// it gives the cached value for unique IDs. NaNs: x86's default NaN
// (0/0 of an empty cluster, zero vectors under cosine) — see x86_nan.
#include "common.h"
#include "exact.h"
#include "kernels.h"

namespace lshkm {

// One thread per centroid: its nearest other centroid (silhouette.hpp:35-56).
__global__ void sil_near_kernel(const double* __restrict__ C, int K, int d, int metric, int32_t* __restrict__ near) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= K) return;
    double mn = -1;
    int arg = 0;
    for (int i = 0; i < K; i++) {
        if (i == c) continue;
        const double dd = exact_dist(C + (size_t)c * d, C + (size_t)i * d, d, metric);
        if (mn == -1 || dd < mn) { mn = dd; arg = i; }
    }
    near[c] = arg;
}

// One thread per member (cluster-sorted order): s(i) (silhouette.hpp:83-144).
// Lanes of a wave mostly share their cluster, so the x_j loads broadcast.
__global__ void sil_point_kernel(const float* __restrict__ X, int d, int metric, const int32_t* __restrict__ rows,
                                 const int64_t* __restrict__ crow, const int32_t* __restrict__ assign,
                                 const int32_t* __restrict__ near, int64_t N, double* __restrict__ s_out) {
    // s_out is indexed by row
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = rows[p];
        const int c = assign[r];
        const float* xi = X + (size_t)r * d;
        const int64_t c0 = crow[c], c1 = crow[c + 1];
        double a = 0.0;
        for (int64_t j = c0; j < c1; j++) a = __dadd_rn(a, exact_dist(xi, X + (size_t)rows[j] * d, d, metric));
        if (c1 - c0 != 1) a = __ddiv_rn(a, (double)(c1 - c0 - 1));
        const int nc = near[c];
        const int64_t n0 = crow[nc], n1 = crow[nc + 1];
        double b = 0.0;
        for (int64_t j = n0; j < n1; j++) b = __dadd_rn(b, exact_dist(xi, X + (size_t)rows[j] * d, d, metric));
        b = x86_nan(__ddiv_rn(b, (double)(n1 - n0)));
        a = x86_nan(a);
        double mx = a;
        if (b > a) mx = b;
        // NaN operands: x86 returns the first NaN operand; both are the default NaN here
        s_out[r] = x86_nan(__ddiv_rn(__dsub_rn(b, a), mx));
    }
}

// One block: per-cluster sums in member order, then the total in cluster order.
constexpr int SIL_SUM_THREADS = 256;
__global__ __launch_bounds__(SIL_SUM_THREADS) void sil_sum_kernel(const double* __restrict__ s, const int32_t* __restrict__ rows,
                                                                 const int64_t* __restrict__ crow, int K, int64_t N,
                                                                 double* __restrict__ raw, double* __restrict__ out) {
    for (int c = threadIdx.x; c < K; c += SIL_SUM_THREADS) {
        double acc = 0.0;
        for (int64_t p = crow[c]; p < crow[c + 1]; p++) acc = __dadd_rn(acc, s[rows[p]]);
        raw[c] = x86_nan(acc);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double tot = 0.0;
        for (int c = 0; c < K; c++) {
            tot = x86_nan(__dadd_rn(tot, raw[c]));
            out[c] = x86_nan(__ddiv_rn(raw[c], (double)(crow[c + 1] - crow[c])));
        }
        out[K] = x86_nan(__ddiv_rn(tot, (double)N));
    }
}

int launch_sil_near(hipStream_t s, const double* C, int K, int d, int metric, int32_t* near) {
    hipLaunchKernelGGL(sil_near_kernel, dim3((K + 63) / 64), dim3(64), 0, s, C, K, d, metric, near);
    return kstatus("sil_near_kernel");
}

int launch_sil_points(hipStream_t s, const float* X, int d, int metric, const int32_t* rows, const int64_t* crow,
                      const int32_t* assign, const int32_t* near, int64_t N, double* s_out) {
    if (N == 0) return 0;
    hipLaunchKernelGGL(sil_point_kernel, dim3(gsz(N, 256, 16384)), dim3(256), 0, s, X, d, metric, rows, crow, assign,
                       near, N, s_out);
    return kstatus("sil_point_kernel");
}

int launch_sil_sum(hipStream_t s, const double* sv, const int32_t* rows, const int64_t* crow, int K, int64_t N,
                   double* raw, double* out) {
    hipLaunchKernelGGL(sil_sum_kernel, dim3(1), dim3(SIL_SUM_THREADS), 0, s, sv, rows, crow, K, N, raw, out);
    return kstatus("sil_sum_kernel");
}

}  // namespace lshkm
