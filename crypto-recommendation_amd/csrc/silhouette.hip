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

// One wave per member i (cluster-sorted order): s(i) (silhouette.hpp:83-144).
// x_i sits in LDS (broadcast reads); lane L evaluates d(x_i, x_j) for member
// j = jb + L of a 64-member batch, then every lane adds the batch's 64
// distances in member order (readlane: the sum stays the reference's sequential
// chain). A thread-per-member form ran one latency-bound chain per lane with too
// few waves to hide it (N / 64 waves).
constexpr int SP_WAVES = 4;
constexpr int SIL_DMAX = 512;

// x_i (LDS) vs x_j (global), rows of fp32 or fp64: the exact.h order, 4-wide
// loads. The whole wave calls it: the squares go through gp_sq_wave (sq: 64 *
// 16 doubles of wave-private LDS; glibc's pow restated for the few squares
// that need it, batched over the wave -- per lane, a wave paid it in nearly
// every term).
template <typename TX, bool EXSQ>
__device__ inline double sil_euclid(const TX* __restrict__ xi, const TX* __restrict__ xj, int d, double* sq) {
    double acc = 0.0;
    int k = 0;
    if ((d & 3) == 0) {
#pragma unroll 1
        for (; k + 8 <= d; k += 8) {
            double a[4], b[4], df[8], p[8];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                ld4d(xi + k + 4 * h, a);
                ld4d(xj + k + 4 * h, b);
#pragma unroll
                for (int u = 0; u < 4; u++) df[4 * h + u] = __dsub_rn(a[u], b[u]);
            }
            gp_sq_wave<8, sizeof(TX) == 8, EXSQ>(df, p, sq);
#pragma unroll
            for (int u = 0; u < 8; u++) acc = __dadd_rn(acc, p[u]);
        }
        if (k < d) {                                        // d % 8 == 4
            double a[4], b[4], df[4], p[4];
            ld4d(xi + k, a);
            ld4d(xj + k, b);
#pragma unroll
            for (int u = 0; u < 4; u++) df[u] = __dsub_rn(a[u], b[u]);
            gp_sq_wave<4, sizeof(TX) == 8, EXSQ>(df, p, sq);
#pragma unroll
            for (int u = 0; u < 4; u++) acc = __dadd_rn(acc, p[u]);
            k += 4;
        }
    }
#pragma unroll 1
    for (; k < d; k++) {
        const double df[1] = {__dsub_rn((double)xi[k], (double)xj[k])};
        double p[1];
        gp_sq_wave<1, sizeof(TX) == 8, EXSQ>(df, p, sq);
        acc = __dadd_rn(acc, p[0]);
    }
    return sqrt(acc);
}

// sum_{j in [j0, j1)} d(x_i, x_rows[j]) in j order (wave-uniform result);
// lanes past j1 repeat the last member so the whole wave stays in step
template <typename TX, bool EXSQ>
__device__ inline double sil_segment(const TX* __restrict__ xi, const TX* __restrict__ X, int d, int metric,
                                     const int32_t* __restrict__ rows, int64_t j0, int64_t j1, int lane,
                                     double* sq) {
    double acc = 0.0;
    for (int64_t jb = j0; jb < j1; jb += 64) {
        const int64_t j = min<int64_t>(jb + lane, j1 - 1);
        const TX* xj = X + (size_t)rows[j] * d;
        const double dj = metric == 0 ? sil_euclid<TX, EXSQ>(xi, xj, d, sq) : exact_dist(xi, xj, d, metric);
        const int n = (int)min<int64_t>(64, j1 - jb);
        for (int t = 0; t < n; t++) acc = __dadd_rn(acc, __shfl(dj, t));
    }
    return acc;
}

// Two members (same cluster) against the same x_j: each x_j load serves both
// (d % 4 == 0).
template <typename TX, bool EXSQ>
__device__ inline void sil_euclid2(const TX* __restrict__ xa, const TX* __restrict__ xb,
                                   const TX* __restrict__ xj, int d, double& da, double& db, double* sq) {
    double aa = 0.0, ab = 0.0;
    int k = 0;
#pragma unroll 1
    for (; k + 8 <= d; k += 8) {
        double df[16], p[16];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            double b[4], u[4], v[4];
            ld4d(xj + k + 4 * h, b);
            ld4d(xa + k + 4 * h, u);
            ld4d(xb + k + 4 * h, v);
#pragma unroll
            for (int e = 0; e < 4; e++) {
                df[8 * h + 2 * e] = __dsub_rn(u[e], b[e]);
                df[8 * h + 2 * e + 1] = __dsub_rn(v[e], b[e]);
            }
        }
        gp_sq_wave<16, sizeof(TX) == 8, EXSQ>(df, p, sq);
#pragma unroll
        for (int e = 0; e < 8; e++) {
            aa = __dadd_rn(aa, p[2 * e]);
            ab = __dadd_rn(ab, p[2 * e + 1]);
        }
    }
    if (k < d) {                                            // d % 8 == 4
        double b[4], u[4], v[4], df[8], p[8];
        ld4d(xj + k, b);
        ld4d(xa + k, u);
        ld4d(xb + k, v);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            df[2 * e] = __dsub_rn(u[e], b[e]);
            df[2 * e + 1] = __dsub_rn(v[e], b[e]);
        }
        gp_sq_wave<8, sizeof(TX) == 8, EXSQ>(df, p, sq);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            aa = __dadd_rn(aa, p[2 * e]);
            ab = __dadd_rn(ab, p[2 * e + 1]);
        }
    }
    da = sqrt(aa);
    db = sqrt(ab);
}

template <typename TX, bool EXSQ>
__device__ inline void sil_segment2(const TX* __restrict__ xa, const TX* __restrict__ xb,
                                    const TX* __restrict__ X, int d, const int32_t* __restrict__ rows, int64_t j0,
                                    int64_t j1, int lane, double& sa, double& sb, double* sq) {
    double acc_a = 0.0, acc_b = 0.0;
    for (int64_t jb = j0; jb < j1; jb += 64) {
        const int64_t j = min<int64_t>(jb + lane, j1 - 1);
        double da, db;
        sil_euclid2<TX, EXSQ>(xa, xb, X + (size_t)rows[j] * d, d, da, db, sq);
        const int n = (int)min<int64_t>(64, j1 - jb);
        for (int t = 0; t < n; t++) {
            acc_a = __dadd_rn(acc_a, __shfl(da, t));
            acc_b = __dadd_rn(acc_b, __shfl(db, t));
        }
    }
    sa = acc_a;
    sb = acc_b;
}

__device__ inline double sil_value(double a, double b, int64_t c0, int64_t c1, int64_t n0, int64_t n1) {
    if (c1 - c0 != 1) a = __ddiv_rn(a, (double)(c1 - c0 - 1));
    b = x86_nan(__ddiv_rn(b, (double)(n1 - n0)));
    a = x86_nan(a);
    double mx = a;
    if (b > a) mx = b;
    // NaN operands: x86 returns the first NaN operand; both are the default NaN here
    return x86_nan(__ddiv_rn(__dsub_rn(b, a), mx));
}

// EXSQ: every difference of the rows squares exactly (data_grid_exact): x*x
// for pow(x, 2) without the per-square test.
template <typename TX, bool EXSQ>
__global__ __launch_bounds__(64 * SP_WAVES) void sil_point_kernel(
    const TX* __restrict__ X, int d, int metric, const int32_t* __restrict__ rows, const int64_t* __restrict__ crow,
    const int32_t* __restrict__ assign, const int32_t* __restrict__ near, int64_t N, double* __restrict__ s_out) {
    __shared__ __attribute__((aligned(16))) TX xs[SP_WAVES][2][SIL_DMAX];
    __shared__ double sqs[SP_WAVES][64 * 16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double* sq = sqs[wave];
    TX* xa = xs[wave][0];
    TX* xb = xs[wave][1];
    // a wave takes members p, p + 1 (cluster-sorted): one pass over the x_j when
    // they share a cluster (euclidean, d % 4 == 0); s_out is indexed by row
    const int64_t npair = (N + 1) / 2;
    for (int64_t q = (int64_t)blockIdx.x * SP_WAVES + wave; q < npair; q += (int64_t)gridDim.x * SP_WAVES) {
        const int64_t p = 2 * q;
        const bool has2 = p + 1 < N;
        const int32_t ra = rows[p], rb = has2 ? rows[p + 1] : ra;
        const int ca = assign[ra], cb = assign[rb];
        __builtin_amdgcn_wave_barrier();                      // previous members' reads of xs are done
        for (int k = lane; k < d; k += 64) {
            xa[k] = X[(size_t)ra * d + k];
            xb[k] = X[(size_t)rb * d + k];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (has2 && ca == cb && metric == 0 && (d & 3) == 0) {
            const int64_t c0 = crow[ca], c1 = crow[ca + 1];
            const int nc = near[ca];
            const int64_t n0 = crow[nc], n1 = crow[nc + 1];
            double a0, a1, b0, b1;
            sil_segment2<TX, EXSQ>(xa, xb, X, d, rows, c0, c1, lane, a0, a1, sq);
            sil_segment2<TX, EXSQ>(xa, xb, X, d, rows, n0, n1, lane, b0, b1, sq);
            if (lane == 0) {
                s_out[ra] = sil_value(a0, b0, c0, c1, n0, n1);
                s_out[rb] = sil_value(a1, b1, c0, c1, n0, n1);
            }
            continue;
        }
        for (int m = 0; m < (has2 ? 2 : 1); m++) {
            const TX* xi = m ? xb : xa;
            const int c = m ? cb : ca;
            const int64_t c0 = crow[c], c1 = crow[c + 1];
            const double a = sil_segment<TX, EXSQ>(xi, X, d, metric, rows, c0, c1, lane, sq);
            const int nc = near[c];
            const int64_t n0 = crow[nc], n1 = crow[nc + 1];
            const double b = sil_segment<TX, EXSQ>(xi, X, d, metric, rows, n0, n1, lane, sq);
            if (lane == 0) s_out[m ? rb : ra] = sil_value(a, b, c0, c1, n0, n1);
        }
    }
}

// d > SIL_DMAX: one thread per member, the same sums.
template <typename TX>
__global__ void sil_point_thread_kernel(const TX* __restrict__ X, int d, int metric, const int32_t* __restrict__ rows,
                                        const int64_t* __restrict__ crow, const int32_t* __restrict__ assign,
                                        const int32_t* __restrict__ near, int64_t N, double* __restrict__ s_out) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = rows[p];
        const int c = assign[r];
        const TX* xi = X + (size_t)r * d;
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

template <typename TX>
static int sil_points_tx(hipStream_t s, const TX* X, int d, int metric, const int32_t* rows, const int64_t* crow,
                         const int32_t* assign, const int32_t* near, int64_t N, double* s_out, bool exsq) {
    if (d > SIL_DMAX) {
        hipLaunchKernelGGL(sil_point_thread_kernel<TX>, dim3(gsz(N, 256, 16384)), dim3(256), 0, s, X, d, metric, rows,
                           crow, assign, near, N, s_out);
        return kstatus("sil_point_thread_kernel");
    }
    if (exsq)
        hipLaunchKernelGGL((sil_point_kernel<TX, true>), dim3(gsz((N + 1) / 2, SP_WAVES, 16384)), dim3(64 * SP_WAVES), 0,
                           s, X, d, metric, rows, crow, assign, near, N, s_out);
    else
        hipLaunchKernelGGL((sil_point_kernel<TX, false>), dim3(gsz((N + 1) / 2, SP_WAVES, 16384)), dim3(64 * SP_WAVES), 0,
                           s, X, d, metric, rows, crow, assign, near, N, s_out);
    return kstatus("sil_point_kernel");
}

int launch_sil_points(hipStream_t s, Pts X, int d, int metric, const int32_t* rows, const int64_t* crow,
                      const int32_t* assign, const int32_t* near, int64_t N, double* s_out, bool exsq) {
    if (N == 0) return 0;
    return X.f64 ? sil_points_tx(s, X.d(), d, metric, rows, crow, assign, near, N, s_out, exsq)
                 : sil_points_tx(s, X.f(), d, metric, rows, crow, assign, near, N, s_out, exsq);
}

int launch_sil_sum(hipStream_t s, const double* sv, const int32_t* rows, const int64_t* crow, int K, int64_t N,
                   double* raw, double* out) {
    hipLaunchKernelGGL(sil_sum_kernel, dim3(1), dim3(SIL_SUM_THREADS), 0, s, sv, rows, crow, K, N, raw, out);
    return kstatus("sil_sum_kernel");
}

}  // namespace lshkm
