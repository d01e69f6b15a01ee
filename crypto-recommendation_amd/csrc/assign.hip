// assign.hip — Lloyd's nearest-centroid assignment on gfx950.
//
// Replaces lloyds_assignment (lib/clustering_phases/assignment.hpp:54-80) with
// CustVector::euclideanDistance (lib/data_structures/cust_vector.hpp:124-136)
// and cosineDistance (:139-155).
//
// Fast path (euclidean): a block owns 128 points (4 waves x 32). Each wave keeps
// its 32 points in registers as the B operand of v_mfma_f32_32x32x2_f32 (lane
// half h holds dims [h*DP/2, (h+1)*DP/2) of point lane&31), centroids stream
// through LDS in chunks of 64 as the A operand, and the accumulator tile
// D[centroid][point] comes out with the point on the lane, so the per-point
// reduction over centroids is register-local. The score is
// s_c = ||c||^2 - 2 x.c; the MFMA result is an f32 FMA chain, so
//   |s~_c - s_c| <= e_c = 2^-24 ((2DP+12) |x||c| + 5 ||c||^2) + 2^-40 (|x|^2+||c||^2)
// covers the chain, the fp32 rounding of c, and the epilogue roundings; the
// 2^-40 term also covers the reference's sequential-fp64 rounding and keeps
// sqrt'ed ties apart. A point is certified when exactly one centroid has
// s~_c - e_c <= min_c (s~_c + e_c); its distance is then recomputed in exact
// reference order (fp64, no FMA contraction: sum_j (x_j - c_j)^2, j = 0..d-1,
// then sqrt). Uncertified points (ties, duplicate centroids, near-ties) go
// to assign_exact_kernel, which evaluates every centroid in reference order
// and keeps the first minimum (strict '<', assignment.hpp:66).
#include "common.h"
#include "kernels.h"
#include "exact.h"

namespace lshkm {

constexpr int AS_THREADS = 256;
constexpr int AS_PB = 128;   // points per block
constexpr int AS_CC = 64;    // centroids per LDS chunk

typedef float floatx16 __attribute__((ext_vector_type(16)));

int assign_dp(int d) {
    const int dps[] = {16, 32, 64, 128, 256};
    for (int dp : dps)
        if (d <= dp) return dp;
    return 0;
}

__global__ void centroid_prep_kernel(const double* __restrict__ C, int K, int Kpad, int d, int DP, int metric,
                                     int xf64, float* __restrict__ C32, float* __restrict__ cconst) {
    // One wave per 64-centroid chunk. cconst = cn2[Kpad] ++ {ecmax, ebmax}[Kpad/64]:
    // the bound coefficients are taken as the max over the chunk, so the MFMA
    // epilogue needs one per-lane bound per chunk instead of per centroid.
    // Cosine (metric 1): cn2[c] = f32(1 / |c|) and the score is -(x.c)/|c|
    // (argmin = the reference's argmin of 1 - cos): |s~ - s| <= (DP + 4) 2^-24 |x|
    // (the f32 chain, c's f32 rounding, 1/|c| and the product's rounding), plus
    // 2^-40 |x| over the reference's last-bit roundings of 1 - ip / denom; a zero
    // centroid (and padding) gets NaN: never taken, never lowers the bound min.
    // fp64 rows (xf64) reach the MFMA rounded to f32: |x_j - f32(x_j)| <= 2^-24 |x_j|
    // + 2^-150, i.e. 2 2^-24 |x||c| more on the euclidean score (2^-24 |x| on the
    // cosine one) plus 2^-150 |c|_1 <= 2^-146 |c| (flushed tiny entries).
    const int c = blockIdx.x * 64 + threadIdx.x;
    const double xw = xf64 ? 2.0 : 0.0;
    float* cn2 = cconst;
    float* chunk = cconst + Kpad + 2 * blockIdx.x;
    double ec = 0.0, eb = 0.0;
    if (c >= K) {
        for (int j = 0; j < DP; j++) C32[(size_t)c * DP + j] = 0.f;
        cn2[c] = metric ? __builtin_nanf("") : __builtin_inff();
    } else {
        double s = 0.0;
        for (int j = 0; j < d; j++) {
            const double v = C[(size_t)c * d + j];
            s = fma(v, v, s);
            C32[(size_t)c * DP + j] = (float)v;
        }
        for (int j = d; j < DP; j++) C32[(size_t)c * DP + j] = 0.f;
        const double up = 1.0 + 0x1p-18;
        const double nc = sqrt(s) * (1.0 + 0x1p-30);
        if (metric == 0) {
            // |c| >= 2^50 (or non-finite) may overflow the f32 chain: no
            // certificate in this call (flag after the chunk bounds)
            cn2[c] = s < 0x1p100 ? (float)s : __builtin_inff();
            if (!(s < 0x1p100)) atomicOr(reinterpret_cast<unsigned int*>(cconst + Kpad + Kpad / 32), 1u);
            ec = 0x1p-24 * (2.0 * DP + 12.0 + xw) * nc * up;
            eb = (0x1p-24 * 5.0 * s + 0x1p-40 * s + (xf64 ? 0x1p-140 * nc : 0.0)) * up + 1e-30;
        } else {
            // 1e-20 <= |c|^2 < 1e30 keeps the f32 chain clear of overflow and of
            // flushed denormals beyond eb ((DP + 4) 2^-124 / |c| for products and
            // c's entries, 2^-116 for x's); outside it,
            // and for a zero centroid 0 (whose NaN the reference's sentinel takes
            // for every row, assignment.hpp:66), eb = inf leaves no certificate
            const bool ok = s >= 1e-20 && s < 1e30;
            const double rc = ok ? 1.0 / sqrt(s) : 0.0;
            cn2[c] = ok ? (float)rc : __builtin_nanf("");
            ec = (0x1p-24 * (DP + 20.0 + xw) + 0x1p-40) * up;
            eb = ok ? ((DP + 4.0) * 0x1p-124 * rc + 0x1p-116) * up
                    : (s == 0.0 && c > 0 ? 0.0 : __builtin_inf());
        }
    }
    for (int off = 32; off >= 1; off >>= 1) {
        ec = fmax(ec, __shfl_xor(ec, off));
        eb = fmax(eb, __shfl_xor(eb, off));
    }
    if (threadIdx.x == 0) {
        chunk[0] = (float)(ec * (1.0 + 0x1p-20));
        chunk[1] = (float)(eb * (1.0 + 0x1p-20));
    }
}

int launch_centroid_prep(hipStream_t s, const double* C, int K, int Kpad, int d, int DP, int metric, bool xf64,
                         float* C32, float* cconst) {
    (void)hipMemsetAsync(cconst + Kpad + Kpad / 32, 0, 4, s);
    hipLaunchKernelGGL(centroid_prep_kernel, dim3((Kpad + 63) / 64), dim3(64), 0, s, C, K, Kpad, d, DP, metric,
                       xf64 ? 1 : 0, C32, cconst);
    return kstatus("assign.hip");
}

template <int DP, int MET, typename TX>
__global__ __launch_bounds__(AS_THREADS, 2) void assign_mfma_kernel(
    const TX* __restrict__ X, int64_t N, int d, const double* __restrict__ C, int Kpad,
    const float* __restrict__ C32, const float* __restrict__ cconst, int32_t* __restrict__ assign,
    double* __restrict__ dist, int32_t* __restrict__ ambig, unsigned long long* __restrict__ ambig_count) {
    constexpr int H = DP / 2;     // dims per lane half
    constexpr int DS = DP + 4;    // padded LDS row stride (floats): conflict-free ds_read_b128
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* lds = reinterpret_cast<float*>(smem);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 31, h = lane >> 5;
    const int64_t pbase = (int64_t)blockIdx.x * AS_PB + wave * 32;

    // ---- phase 0: this wave's 32 rows -> LDS -> registers (B operand)
    float* xs = lds + wave * 32 * DS;
    if (d == DP) {
        for (int e4 = lane; e4 < 32 * DP / 4; e4 += 64) {
            const int r = e4 / (DP / 4), j = (e4 % (DP / 4)) * 4;
            const int64_t row = pbase + r;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (sizeof(TX) == 4) {
                if (row < N) v = *reinterpret_cast<const float4*>(X + row * DP + j);
            } else if (row < N) {
                const double2 a = *reinterpret_cast<const double2*>(X + row * DP + j);
                const double2 b = *reinterpret_cast<const double2*>(X + row * DP + j + 2);
                v = make_float4((float)a.x, (float)a.y, (float)b.x, (float)b.y);
            }
            *reinterpret_cast<float4*>(xs + r * DS + j) = v;
        }
    } else if (sizeof(TX) == 8 && (d & 1) == 0) {
        // fp64 rows of even d (the recommender's user vectors, d = number of coins):
        // 16-B loads, a row per 64-lane pass (was one 8-B load per element)
        for (int e2 = lane; e2 < 32 * DP / 2; e2 += 64) {
            const int r = e2 / (DP / 2), j = (e2 % (DP / 2)) * 2;
            const int64_t row = pbase + r;
            float2 v = make_float2(0.f, 0.f);
            if (row < N && j < d) {
                const double2 a = *reinterpret_cast<const double2*>(X + row * d + j);
                v = make_float2((float)a.x, (float)a.y);
            }
            *reinterpret_cast<float2*>(xs + r * DS + j) = v;
        }
    } else if (sizeof(TX) == 4 && (d & 3) == 0) {
        for (int e4 = lane; e4 < 32 * DP / 4; e4 += 64) {
            const int r = e4 / (DP / 4), j = (e4 % (DP / 4)) * 4;
            const int64_t row = pbase + r;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (row < N && j < d) v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(X) + row * d + j);
            *reinterpret_cast<float4*>(xs + r * DS + j) = v;
        }
    } else {
        for (int e = lane; e < 32 * DP; e += 64) {
            const int r = e / DP, j = e % DP;
            const int64_t row = pbase + r;
            xs[r * DS + j] = (row < N && j < d) ? (float)X[row * d + j] : 0.f;
        }
    }
    __syncthreads();
    float b[H];
#pragma unroll
    for (int s = 0; s < H; s += 4) {
        const float4 v = *reinterpret_cast<const float4*>(xs + col * DS + h * H + s);
        b[s] = v.x; b[s + 1] = v.y; b[s + 2] = v.z; b[s + 3] = v.w;
    }
    double xn2 = 0.0;
#pragma unroll
    for (int s = 0; s < H; s++) xn2 = fma((double)b[s], (double)b[s], xn2);
    xn2 += __shfl_xor(xn2, 32);
    if (sizeof(TX) == 8) xn2 = xn2 * (1.0 + 0x1p-21) + 0x1p-280;   // |x|^2 from the f32-rounded row: still an upper bound
    const float nx = (float)(sqrt(xn2) * (1.0 + 0x1p-30));
    // cosine: |x| >= 1e18 may overflow the f32 products (|c| < 1e15 is checked
    // in the prep): no certificate, the row goes to the exact pass
    // |x| >= 2^50 (euclidean) / 1e18 (cosine) may overflow the f32 products: no
    // certificate, the row goes to the exact pass (false for inf / nan too)
    const float ex = MET == 0 ? (xn2 < 0x1p100 ? (float)(0x1p-40 * xn2 * (1.0 + 0x1p-18) + 1e-30) : __builtin_inff())
                              : (xn2 < 1e36 ? 0.f : __builtin_inff());
    __syncthreads();   // LDS now reused for centroid chunks

    float L1 = __builtin_inff(), L2 = __builtin_inff(), U = __builtin_inff();
    int i1 = 0;
    float* cs = lds;                 // [64][DS]
    float* cc = lds + AS_CC * DS;    // [64] cn2 of the chunk
    const float* chunkc = cconst + Kpad;
    for (int c0 = 0; c0 < Kpad; c0 += AS_CC) {
        for (int e4 = threadIdx.x; e4 < AS_CC * DP / 4; e4 += AS_THREADS) {
            const int r = e4 / (DP / 4), j = (e4 % (DP / 4)) * 4;
            *reinterpret_cast<float4*>(cs + r * DS + j) =
                *reinterpret_cast<const float4*>(C32 + (size_t)(c0 + r) * DP + j);
        }
        if (threadIdx.x < AS_CC) cc[threadIdx.x] = cconst[c0 + threadIdx.x];
        const float E = fmaf(nx, chunkc[2 * (c0 / AS_CC)], chunkc[2 * (c0 / AS_CC) + 1] + ex);
        __syncthreads();
#pragma unroll 1
        for (int t = 0; t < AS_CC / 32; t++) {
            floatx16 acc;
#pragma unroll
            for (int r = 0; r < 16; r++) acc[r] = 0.f;
            const float* arow = cs + (t * 32 + col) * DS + h * H;
#pragma unroll
            for (int s = 0; s < H; s += 4) {
                const float4 a = *reinterpret_cast<const float4*>(arow + s);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b[s], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b[s + 1], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b[s + 2], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b[s + 3], acc, 0, 0, 0);
            }
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int cb = t * 32 + 8 * g + 4 * h;   // D rows of registers 4g..4g+3
                const float4 cn = *reinterpret_cast<const float4*>(cc + cb);
                const float cnv[4] = {cn.x, cn.y, cn.z, cn.w};
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float sc = MET == 0 ? fmaf(-2.f, acc[4 * g + q], cnv[q]) : -acc[4 * g + q] * cnv[q];
                    const float lo = sc - E, hi = sc + E;
                    if (lo < L1) { L2 = L1; L1 = lo; i1 = c0 + cb + q; }
                    else if (lo < L2) L2 = lo;
                    U = fminf(U, hi);
                }
            }
        }
        __syncthreads();
    }

    // ---- merge the two lane halves that share a point
    const float oL1 = __shfl_xor(L1, 32), oL2 = __shfl_xor(L2, 32), oU = __shfl_xor(U, 32);
    const int oi1 = __shfl_xor(i1, 32);
    float nL2; int ni1;
    if (oL1 < L1 || (oL1 == L1 && oi1 < i1)) { ni1 = oi1; nL2 = fminf(L1, oL2); }
    else { ni1 = i1; nL2 = fminf(oL1, L2); }
    U = fminf(U, oU);
    const bool cbad = __float_as_uint(cconst[Kpad + Kpad / 32]) != 0u;   // centroid out of the f32 range
    const bool cert = !cbad && nL2 > U;
    const int64_t row = pbase + col;
    const bool valid = row < N;

    // ---- exact-order distance of the certified winner: lanes h=0 sum dims
    // [0,H), hand the partial to lane h=1, which sums [H,2H) (j ascending).
    if (MET == 1) {
        // cosine (metric.hpp cosine distance): exact.h's certified fast form,
        // soft-x87 for the rows it cannot certify
        // soft-x87 for the rows it cannot certify, listed (after the ambiguous
        // rows' half of the list) for cos_fix_kernel: inline, one failing lane
        // would make its whole wave pay the soft chain
        bool fix = false;
        if (h == 1 && valid) {
            if (cert) {
                assign[row] = ni1;
                double v;
                if (cosine_fast(X + row * d, C + (size_t)ni1 * d, d, v)) dist[row] = v;
                else fix = true;
            } else {
                const unsigned long long slot = atomicAdd(ambig_count, 1ull);
                ambig[slot] = (int32_t)row;
            }
        }
        const unsigned long long fb = __ballot(fix);
        if (fb) {
            const int leader = __builtin_ctzll(fb);
            unsigned long long base = 0;
            if (lane == leader) base = atomicAdd(ambig_count + 1, (unsigned long long)__popcll(fb));
            base = __shfl(base, leader);
            if (fix) ambig[N + base + __popcll(fb & ((1ull << lane) - 1ull))] = (int32_t)row;
        }
        return;
    }
    double accd = 0.0;
    const TX* xrow = X + (valid ? row : 0) * d;
    if (h == 0 && cert && valid) {
        const double* crow = C + (size_t)ni1 * d;
#pragma unroll
        for (int s = 0; s < H; s++)
            if (s < d) {
                const double xv = sizeof(TX) == 4 ? (double)b[s] : (double)xrow[s];
                const double df = __dsub_rn(xv, crow[s]);
                accd = __dadd_rn(accd, gp_sq(df));
            }
    }
    const double part = __shfl_xor(accd, 32);
    if (h == 1 && valid) {
        if (cert) {
            double a2 = part;
            const double* crow = C + (size_t)ni1 * d;
#pragma unroll
            for (int s = 0; s < H; s++)
                if (H + s < d) {
                    const double xv = sizeof(TX) == 4 ? (double)b[s] : (double)xrow[H + s];
                    const double df = __dsub_rn(xv, crow[H + s]);
                    a2 = __dadd_rn(a2, gp_sq(df));
                }
            assign[row] = ni1;
            dist[row] = sqrt(a2);
        } else {
            const unsigned long long slot = atomicAdd(ambig_count, 1ull);
            ambig[slot] = (int32_t)row;
        }
    }
}

template <typename TX>
static int assign_mfma_tx(hipStream_t s, const TX* X, int64_t N, int d, int DP, const double* C, int Kpad, int metric,
                          const float* C32, const float* cconst, int32_t* assign, double* dist, int32_t* ambig,
                          unsigned long long* ambig_count) {
    const dim3 grid((unsigned)((N + AS_PB - 1) / AS_PB)), block(AS_THREADS);
    const size_t lds = (size_t)4 * 32 * (DP + 4) * 4;   // >= chunk (64*(DP+4) + 192) floats
    switch (DP * 2 + (metric ? 1 : 0)) {
#define AS_CASE(V) \
        case 2 * V: hipLaunchKernelGGL((assign_mfma_kernel<V, 0, TX>), grid, block, lds, s, X, N, d, C, Kpad, C32, cconst, assign, dist, ambig, ambig_count); break; \
        case 2 * V + 1: hipLaunchKernelGGL((assign_mfma_kernel<V, 1, TX>), grid, block, lds, s, X, N, d, C, Kpad, C32, cconst, assign, dist, ambig, ambig_count); break;
        AS_CASE(16) AS_CASE(32) AS_CASE(64) AS_CASE(128) AS_CASE(256)
#undef AS_CASE
        default: return -4;
    }
    return kstatus("assign.hip");
}

int launch_assign_mfma(hipStream_t s, Pts X, int64_t N, int d, int DP, const double* C, int K, int Kpad, int metric,
                       const float* C32, const float* cconst, int32_t* assign, double* dist, int32_t* ambig,
                       unsigned long long* ambig_count) {
    (void)K;
    if (N <= 0) return 0;
    return X.f64 ? assign_mfma_tx(s, X.d(), N, d, DP, C, Kpad, metric, C32, cconst, assign, dist, ambig, ambig_count)
                 : assign_mfma_tx(s, X.f(), N, d, DP, C, Kpad, metric, C32, cconst, assign, dist, ambig, ambig_count);
}

// Certified cosine winners whose distance IpAcc could not certify: one lane
// per listed row, the soft-x87 chain (exact.h exact_cosine_x87).
template <typename TX>
__global__ __launch_bounds__(256) void cos_fix_kernel(const TX* __restrict__ X, int d, const double* __restrict__ C,
                                                      const int32_t* __restrict__ rows,
                                                      const unsigned long long* __restrict__ count,
                                                      const int32_t* __restrict__ assign, double* __restrict__ dist) {
    const int64_t n = (int64_t)*count;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int64_t row = rows[i];
        dist[row] = exact_cosine_x87(X + row * d, C + (size_t)assign[row] * d, d);
    }
}

int launch_cos_fix(hipStream_t s, Pts X, int64_t N, int d, const double* C, const int32_t* rows,
                   const unsigned long long* count, const int32_t* assign, double* dist) {
    if (N <= 0) return 0;
    const dim3 grid((unsigned)std::min<int64_t>((N + 255) / 256, 2048));
    if (X.f64) hipLaunchKernelGGL(cos_fix_kernel<double>, grid, dim3(256), 0, s, X.d(), d, C, rows, count, assign, dist);
    else hipLaunchKernelGGL(cos_fix_kernel<float>, grid, dim3(256), 0, s, X.f(), d, C, rows, count, assign, dist);
    return kstatus("assign.hip");
}

// ---------------------------------------------------------------- exact pass
constexpr int XC_MAXV = 4;   // cosine candidate form: K <= 256 (values kept per lane)
constexpr int XE_SPLIT = 2;  // blocks per list segment (segmented form)
// One wave per listed row; lane c evaluates centroids c, c+64, ... in the
// reference's exact order (exact.h); the first minimum wins.
template <typename TX>
__global__ __launch_bounds__(256) void assign_exact_kernel(
    const TX* __restrict__ X, int64_t N, int d, const double* __restrict__ C, int K, int metric,
    const int32_t* __restrict__ rows, const unsigned long long* __restrict__ row_count, int64_t max_rows,
    int32_t* __restrict__ assign, double* __restrict__ dist, const int32_t* __restrict__ seg_counts,
    int64_t seg_rows, const double* __restrict__ xn2, const double* __restrict__ nbv) {
    const int lane = threadIdx.x & 63;
    int64_t wglobal = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    int64_t nw = (int64_t)gridDim.x * 4;
    int64_t total = rows ? (int64_t)*row_count : N;
    if (seg_counts) {            // XE_SPLIT blocks per segment of the persistent fused form's list
        const int seg = blockIdx.x % (gridDim.x / XE_SPLIT);   // segments across XCDs (cos_fix_seg_kernel)
        rows += (int64_t)seg * seg_rows;
        total = seg_counts[2 * seg];
        wglobal = (int64_t)(blockIdx.x / (gridDim.x / XE_SPLIT)) * 4 + (threadIdx.x >> 6);
        nw = XE_SPLIT * 4;
    }
    if (total > max_rows) total = max_rows;
    for (int64_t it = wglobal; it < total; it += nw) {
        const int64_t row = rows ? rows[it] : it;
        const TX* x = X + row * d;
        double best = 0.0; int bi = -1;
        // cosine: the row's / centroids' sums of squares precomputed (row_sumsq,
        // the prep's nbv; glibc pow per square, the same for every pair) when given
        const double xa = metric == 1 && xn2 ? xn2[row] : -1.0;
        if (metric == 1 && K <= 64 * XC_MAXV) {
            // cosine: certified values (exact.h cosine_interval) for every
            // centroid, the soft-x87 chain only for those whose interval can
            // still reach the minimum; a row with an unknown value (zero
            // vectors, NaN/inf, extreme ranges) takes the full soft pass below
            double v[XC_MAXV], rad[XC_MAXV];
            int st[XC_MAXV];
            double U = __builtin_inf();
            bool unknown = false;
#pragma unroll
            for (int k = 0; k < XC_MAXV; k++) {
                const int c = lane + 64 * k;
                st[k] = 0; v[k] = 0.0; rad[k] = 0.0;
                if (c < K) {
                    st[k] = cosine_interval(x, C + (size_t)c * d, d, v[k], rad[k], xa, nbv ? nbv[c] : -1.0);
                    unknown |= st[k] == 2;
                    if (st[k] != 2) U = fmin(U, v[k] + rad[k]);
                }
            }
            if (!__ballot(unknown)) {
                for (int off = 32; off >= 1; off >>= 1) U = fmin(U, __shfl_xor(U, off));
#pragma unroll
                for (int k = 0; k < XC_MAXV; k++) {
                    const int c = lane + 64 * k;
                    if (c < K && v[k] - rad[k] <= U) {     // non-candidates are strictly above the minimum
                        const double dd = st[k] == 0 ? v[k] : exact_cosine_x87(x, C + (size_t)c * d, d, xa, nbv ? nbv[c] : -1.0);
                        if (bi < 0 || dd < best) { best = dd; bi = c; }
                    }
                }
                for (int off = 32; off >= 1; off >>= 1) {
                    const double ob = __shfl_xor(best, off);
                    const int oi = __shfl_xor(bi, off);
                    const bool take = oi >= 0 && (bi < 0 || ob < best || (ob == best && oi < bi));
                    if (take) { best = ob; bi = oi; }
                }
                if (lane == 0) {
                    assign[row] = bi;
                    dist[row] = best;
                }
                continue;
            }
        }
        for (int c = lane; c < K; c += 64) {
            const double dd = metric == 0 ? exact_euclid(x, C + (size_t)c * d, d)
                                          : exact_cosine_x87(x, C + (size_t)c * d, d, xa, nbv ? nbv[c] : -1.0);
            // assignment.hpp:66: the -1 sentinel takes centroid 0's distance even
            // if NaN (a zero vector under cosine), which then blocks every later
            // '<'; any other NaN is never taken
            if (bi < 0 ? (dd == dd || c == 0) : dd < best) { best = dd; bi = c; }
        }
        // wave argmin: smallest value, then smallest index (= first strict minimum in c order)
        for (int off = 32; off >= 1; off >>= 1) {
            const double ob = __shfl_xor(best, off);
            const int oi = __shfl_xor(bi, off);
            const bool take = oi >= 0 && (bi < 0 || ob < best || (ob == best && oi < bi));
            if (take) { best = ob; bi = oi; }
        }
        if (lane == 0) {
            assign[row] = bi < 0 ? 0 : bi;
            dist[row] = bi < 0 ? -1.0 : best;
        }
    }
}

int launch_assign_exact(hipStream_t s, Pts X, int64_t N, int d, const double* C, int K, int metric,
                        const int32_t* rows, const unsigned long long* row_count, int64_t max_rows,
                        int32_t* assign, double* dist, const int32_t* seg_counts, int64_t seg_rows, int nseg,
                        const double* xn2, const double* nbv) {
    if (max_rows <= 0) return 0;
    // rows == NULL: every row (fallback path); else a device-counted list that is
    // usually ~0.3% of the rows: one block per CU, waves loop over the list.
    const int64_t blocks = seg_counts ? (int64_t)nseg * XE_SPLIT : std::min<int64_t>((max_rows + 3) / 4, rows ? 256 : 2048);
    if (blocks <= 0) return 0;
    if (X.f64)
        hipLaunchKernelGGL(assign_exact_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, s, X.d(), N, d, C, K,
                           metric, rows, row_count, max_rows, assign, dist, seg_counts, seg_rows, xn2, nbv);
    else
        hipLaunchKernelGGL(assign_exact_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s, X.f(), N, d, C, K,
                           metric, rows, row_count, max_rows, assign, dist, seg_counts, seg_rows, xn2, nbv);
    return kstatus("assign.hip");
}

// Listed (uncertified) rows, euclidean: the same reference-order distances as
// assign_exact_kernel, but a wave takes XB_R rows at once against a transposed
// fp64 copy CT[j][c], so each centroid value is loaded once (coalesced, lane =
// centroid) for XB_R rows. Lane holds centroids c0 + lane + 64i, i < 4.
constexpr int XB_R = 8;
constexpr int XB_WAVES = 4;
constexpr int XB_SPLIT = 4;      // blocks per list segment: 16 waves per CU hide the CT-load latency
constexpr int XB_DMAX = 256;

__global__ void transpose_centroids_kernel(const double* __restrict__ C, int K, int Kpad, int d,
                                           double* __restrict__ CT) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)d * Kpad) return;
    const int j = (int)(e / Kpad), c = (int)(e % Kpad);
    CT[e] = c < K ? C[(size_t)c * d + j] : 0.0;
}

template <typename TX>
__global__ __launch_bounds__(64 * XB_WAVES) void assign_exact_batch_kernel(
    const TX* __restrict__ X, int d, const double* __restrict__ CT, int K, int Kpad,
    const int32_t* __restrict__ rows, const unsigned long long* __restrict__ row_count, int64_t max_rows,
    int32_t* __restrict__ assign, double* __restrict__ dist, const int32_t* __restrict__ seg_counts,
    int64_t seg_rows) {
    __shared__ TX xs[XB_WAVES][XB_R][XB_DMAX];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t total, g0, gstride;
    if (seg_counts) {            // XB_SPLIT blocks per segment (the one persistent block b wrote)
        const int nseg = gridDim.x / XB_SPLIT;   // segments across XCDs (cos_fix_seg_kernel)
        const int seg = blockIdx.x % nseg, part = blockIdx.x / nseg;
        rows += (int64_t)seg * seg_rows;
        total = seg_counts[2 * seg];
        g0 = (int64_t)part * XB_WAVES + wave;
        gstride = (int64_t)XB_SPLIT * XB_WAVES;
    } else {
        total = (int64_t)*row_count;
        if (total > max_rows) total = max_rows;
        g0 = (int64_t)blockIdx.x * XB_WAVES + wave;
        gstride = (int64_t)gridDim.x * XB_WAVES;
    }
    const int64_t ngroups = (total + XB_R - 1) / XB_R;
    for (int64_t g = g0; g < ngroups; g += gstride) {
        const int nr = (int)min((int64_t)XB_R, total - g * XB_R);
        int64_t myrow[XB_R];
#pragma unroll
        for (int r = 0; r < XB_R; r++) myrow[r] = rows[g * XB_R + min(r, nr - 1)];   // pad with the last row
#pragma unroll
        for (int r = 0; r < XB_R; r++)
            for (int j = lane; j < d; j += 64) xs[wave][r][j] = X[myrow[r] * d + j];
        wave_sync();
        double best[XB_R];
        int bi[XB_R];
#pragma unroll
        for (int r = 0; r < XB_R; r++) { best[r] = 0.0; bi[r] = -1; }
        for (int c0 = 0; c0 < K; c0 += 256) {
            double acc[XB_R][4];
#pragma unroll
            for (int r = 0; r < XB_R; r++)
#pragma unroll
                for (int i = 0; i < 4; i++) acc[r][i] = 0.0;
            const double* ct = CT + c0 + lane;   // CT rows are padded to a multiple of 256 columns
#pragma unroll 4
            for (int j = 0; j < d; j++) {
                double cv[4];
#pragma unroll
                for (int i = 0; i < 4; i++) cv[i] = ct[(size_t)j * Kpad + 64 * i];
#pragma unroll
                for (int r = 0; r < XB_R; r++) {
                    const double xj = (double)xs[wave][r][j];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const double df = __dsub_rn(xj, cv[i]);
                        acc[r][i] = __dadd_rn(acc[r][i], gp_sq(df));
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {           // increasing c: strict '<' keeps the first minimum
                const int c = c0 + lane + 64 * i;
                if (c >= K) continue;
#pragma unroll
                for (int r = 0; r < XB_R; r++) {
                    const double dd = sqrt(acc[r][i]);
                    if (bi[r] < 0 || dd < best[r]) { best[r] = dd; bi[r] = c; }
                }
            }
        }
#pragma unroll
        for (int r = 0; r < XB_R; r++) {
            double b = best[r];
            int i1 = bi[r];
            for (int off = 32; off >= 1; off >>= 1) {
                const double ob = __shfl_xor(b, off);
                const int oi = __shfl_xor(i1, off);
                const bool take = oi >= 0 && (i1 < 0 || ob < b || (ob == b && oi < i1));
                if (take) { b = ob; i1 = oi; }
            }
            if (lane == 0 && r < nr) {
                assign[myrow[r]] = i1;
                dist[myrow[r]] = b;
            }
        }
        wave_sync();
    }
}

// ------------------------------------------------------- pruned exact pass
// Listed rows, euclidean, K <= 256 (the persistent fused form's lists): a wave
// takes XB_R rows; phase 1 scores every centroid in f32 (an FMA chain over a
// transposed f32 copy CT32[j][c], loaded once per XB_R rows) with the bound e_c
// of the f32 path above; the candidates are the centroids with
// s~_c - e_c <= min (s~ + e) -- every other centroid's reference distance is
// provably larger than some candidate's -- and phase 2 evaluates only those in
// the reference's exact order (one lane each), keeping the first minimum.
// A row whose f32 scores are not all finite, or with more than 64 candidates,
// evaluates every centroid exactly instead.
#ifndef XP_ROWS
#define XP_ROWS 8
#endif
#ifndef XP_SPLITS
#define XP_SPLITS 4
#endif
constexpr int XP_R = XP_ROWS;
#ifndef XP_WIDE_ROWS
#define XP_WIDE_ROWS 2      // rows per wave at 256 < K <= 1024 (16 chunks of 64 centroids)
#endif
constexpr int XP_WR = XP_WIDE_ROWS;
constexpr int XP_WAVES = 4;
constexpr int XP_SPLIT = XP_SPLITS;

// The reference's distance of one (row, centroid) pair on the pruned pass:
// euclidean in exact order; cosine by the soft-x87 chain (16-B loads when the
// row length allows).
// The reference's euclidean chain with glibc's pow per square, a rolled loop
// inlined where it is used: the kernels' rare exact paths (a call would raise
// the whole kernel to the calling convention's 256 VGPRs).
template <typename TX>
__device__ __attribute__((always_inline)) inline double exact_euclid_rolled(const TX* __restrict__ x,
                                                                            const double* __restrict__ c, int d) {
    double acc = 0.0;
#pragma unroll 1
    for (int j = 0; j < d; j++) acc = __dadd_rn(acc, gp_sq(__dsub_rn((double)x[j], c[j])));
    return sqrt(acc);
}

template <int MET, typename TX>
__device__ inline double pruned_dist(const TX* __restrict__ x, const double* __restrict__ c, int d) {
    if constexpr (MET == 0) {
        return exact_euclid_rolled(x, c, d);
    } else {
        if constexpr (sizeof(TX) == 4) {
            if ((d & 15) == 0) return exact_cosine_x87_b16(x, c, d);
        }
        return exact_cosine_x87(x, c, d);
    }
}

// The squared euclidean chain of one (row, centroid) pair in the reference's
// order with x*x squares: the reference's value unless pw.hard() afterwards
// (some square pow(x, 2) may round differently, gpow2.h).
template <typename TX>
__device__ inline double euclid_sumsq_mul(const TX* __restrict__ x, const double* __restrict__ c, int d, PwAcc& pw) {
    double acc = 0.0;
    for (int j0 = 0; j0 < d; j0 += 16) {
        double cv[16];
#pragma unroll
        for (int t = 0; t < 16; t++) cv[t] = j0 + t < d ? c[j0 + t] : 0.0;
#pragma unroll
        for (int t = 0; t < 16; t++)
            if (j0 + t < d) {
                const double df = __dsub_rn((double)x[j0 + t], cv[t]);
                const double p = __dmul_rn(df, df);
                pw.add<true>(df);
                acc = __dadd_rn(acc, p);
            }
    }
    return acc;
}

// (best, bi) over a group of G lanes (xor offsets < G): the smallest value, the
// first index on ties (assignment.hpp:66-69 strict '<' in index order); bi < 0:
// no candidate in the lane.
template <int G>
__device__ inline void group_argmin(double& best, int& bi) {
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) {
        const double ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(bi, off);
        const bool take = oi >= 0 && (bi < 0 || ob < best || (ob == best && oi < bi));
        if (take) { best = ob; bi = oi; }
    }
}
template <int G>
__device__ inline double group_min(double v) {
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) v = fmin(v, __shfl_xor(v, off));
    return v;
}

// The pruned pass's euclidean pick among a group's candidates (lane: centroid c,
// or c < 0). The chains run with x*x squares; where one of the group holds a
// square pow may round differently (PwAcc), each chain is within 2^-43 of the
// reference's (both sums' roundings, <= gamma_255 of the non-negative terms, plus
// one ulp per square), so the x*x winner stands when every other candidate's sum
// exceeds its own by 2^-41 relative -- the reference's sums then order the same
// way and their square roots are distinct doubles. Otherwise every chain is
// redone with pow (gp_sq). exact_dist (LSHKM_DIST_EXACT): the winner's distance
// from its pow chain; certified mode keeps the x*x one (2^-44 relative).
template <int G, typename TX>
__device__ inline void pruned_pick_euclid(const TX* __restrict__ xr, const double* __restrict__ C, int d, int c,
                                          bool exact_dist, double& best, int& bi) {
    PwAcc pw;
    const double S = c >= 0 ? euclid_sumsq_mul(xr, C + (size_t)c * d, d, pw) : 0.0;
    const bool hard = c >= 0 && pw.hard();
    best = c >= 0 ? sqrt(S) : 0.0;
    bi = c;
    group_argmin<G>(best, bi);
    int anyh = hard ? 1 : 0;
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) anyh |= __shfl_xor(anyh, off);
    if (!anyh) return;                                           // every chain is pow's
    const double S1 = group_min<G>(c >= 0 && c == bi ? S : __builtin_inf());
    const double S2 = group_min<G>(c >= 0 && c != bi ? S : __builtin_inf());
    if (S2 != __builtin_inf() && !(S2 - S1 > 0x1p-41 * S2)) {      // S2 = inf: the lone candidate
        // too close to call: the reference's chains
        best = c >= 0 ? exact_euclid_rolled(xr, C + (size_t)c * d, d) : 0.0;
        bi = c;
        group_argmin<G>(best, bi);
        return;
    }
    if (!exact_dist) return;
    const int w = bi;
    double v = __builtin_inf();
    if (c == w) v = hard ? exact_euclid_rolled(xr, C + (size_t)c * d, d) : best;
    best = group_min<G>(v);
}

__global__ void exact_prep_kernel(const double* __restrict__ C, int K, int Kpad, int d, int xf64,
                                  float* __restrict__ CT32, float* __restrict__ cconst, int metric) {
    // one wave per centroid: CT32 [d][Kpad], cconst = cn2[Kpad] ++ {ec, eb}[Kpad/64]
    // (chunk maxima by atomicMax on the bits of positive floats; zeroed first).
    // cosine: CT32 holds the normalised row (score -x.c^), cconst 0, or +inf for
    // a zero / extreme-norm centroid (rows then evaluate every centroid exactly)
    const int c = blockIdx.x, lane = threadIdx.x;
    double scale = 1.0;
    if (metric == 1) {
        double q = 0.0;
        for (int j = lane; j < d; j += 64) {
            const double v = c < K ? C[(size_t)c * d + j] : 0.0;
            q = fma(v, v, q);
        }
        for (int off = 32; off >= 1; off >>= 1) q += __shfl_xor(q, off);
        scale = (q >= 1e-200 && q <= 1e200) ? 1.0 / sqrt(q) : 0.0;
        if (c < K && scale == 0.0) {
            for (int j = lane; j < d; j += 64) CT32[(size_t)j * Kpad + c] = 0.f;
            if (lane == 0) cconst[c] = __builtin_inff();
            return;
        }
    }
    double sq = 0.0;
    for (int j = lane; j < d; j += 64) {
        const double v = c < K ? C[(size_t)c * d + j] * scale : 0.0;
        sq = fma(v, v, sq);
        CT32[(size_t)j * Kpad + c] = (float)v;
    }
    for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off);
    if (lane != 0) return;
    if (c >= K) { cconst[c] = __builtin_inff(); return; }
    if (metric == 1) {
        // |s~ - x.c^| <= (d + 2) 2^-24 |x| (f32 FMA chain, c^'s f32 rounding), and
        // the reference's q = x.c / (|x||c|) sits within 2^-40 |x| of x.c^ / |x| . |x|
        cconst[c] = 0.f;
        const double ec = ((d + 2.0) * 0x1p-24 * (1.0 + 0x1p-10) + 0x1p-40 + (xf64 ? 0x1p-23 : 0.0)) * (1.0 + 0x1p-18);
        unsigned int* chunk = reinterpret_cast<unsigned int*>(cconst + Kpad + 2 * (c / 64));
        atomicMax(chunk, __float_as_uint((float)(ec * (1.0 + 0x1p-20))));
        atomicMax(chunk + 1, __float_as_uint(1e-30f));
        return;
    }
    const double up = 1.0 + 0x1p-18;
    const double nc = sqrt(sq) * (1.0 + 0x1p-30);
    cconst[c] = (float)sq;
    // fp64 rows are scored from their f32 roundings (as centroid_prep_kernel)
    const double ec = 0x1p-24 * (2.0 * d + 12.0 + (xf64 ? 2.0 : 0.0)) * nc * up;
    const double eb = (0x1p-24 * 5.0 * sq + 0x1p-40 * sq + (xf64 ? 0x1p-140 * nc : 0.0)) * up + 1e-30;
    unsigned int* chunk = reinterpret_cast<unsigned int*>(cconst + Kpad + 2 * (c / 64));
    atomicMax(chunk, __float_as_uint((float)(ec * (1.0 + 0x1p-20))));
    atomicMax(chunk + 1, __float_as_uint((float)(eb * (1.0 + 0x1p-20))));
}

// NCH = Kpad / 64 centroid chunks scored per lane (K <= 64 NCH), R rows per wave.
template <typename TX, int NCH = 4, int R = XP_R, int MET = 0>
__global__ __launch_bounds__(64 * XP_WAVES) void assign_pruned_kernel(
    const TX* __restrict__ X, int d, const double* __restrict__ C, const float* __restrict__ CT32,
    const float* __restrict__ cconst, int K, int Kpad, const int32_t* __restrict__ rows,
    const unsigned long long* __restrict__ row_count, int64_t max_rows, int32_t* __restrict__ assign,
    double* __restrict__ dist, const int32_t* __restrict__ seg_counts, int64_t seg_rows, int exact_dist) {
    constexpr int RL = 64 / R;           // lanes per row in the candidate phase
    __shared__ TX xs[XP_WAVES][R][XB_DMAX];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t total, g0, gstride;
    if (seg_counts) {
        const int nseg = gridDim.x / XP_SPLIT;   // segments across XCDs (cos_fix_seg_kernel)
        const int seg = blockIdx.x % nseg, part = blockIdx.x / nseg;
        rows += (int64_t)seg * seg_rows;
        total = seg_counts[2 * seg];
        g0 = (int64_t)part * XP_WAVES + wave;
        gstride = (int64_t)XP_SPLIT * XP_WAVES;
    } else {
        total = (int64_t)*row_count;
        if (total > max_rows) total = max_rows;
        g0 = (int64_t)blockIdx.x * XP_WAVES + wave;
        gstride = (int64_t)gridDim.x * XP_WAVES;
    }
    const float* chunkc = cconst + Kpad;
    const int64_t ngroups = (total + R - 1) / R;
    for (int64_t g = g0; g < ngroups; g += gstride) {
        const int nr = (int)min((int64_t)R, total - g * R);
        int32_t myrow[R];
#pragma unroll
        for (int r = 0; r < R; r++) myrow[r] = rows[g * R + min(r, nr - 1)];   // pad with the last row
        // every row value of the group in flight at once (d <= XB_DMAX: at most
        // XB_DMAX / 64 per lane and row), then staged in LDS
        float xn2p[R];
        TX xv[R][XB_DMAX / 64];
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int u = 0; u < XB_DMAX / 64; u++) {
                const int j = lane + 64 * u;
                xv[r][u] = j < d ? X[(int64_t)myrow[r] * d + j] : TX(0);
            }
#pragma unroll
        for (int r = 0; r < R; r++) {
            float q = 0.f;
#pragma unroll
            for (int u = 0; u < XB_DMAX / 64; u++) {
                const int j = lane + 64 * u;
                if (j < d) {
                    xs[wave][r][j] = xv[r][u];
                    q = fmaf((float)xv[r][u], (float)xv[r][u], q);
                }
            }
            xn2p[r] = q;
        }
        wave_sync();
        // phase 1: f32 scores of centroids c = lane + 64 i
        float acc[R][NCH];
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int i = 0; i < NCH; i++) acc[r][i] = 0.f;
        // chunks past Kpad read chunk 0 (their scores are never used): the loads
        // carry no branch, so the unrolled iterations' loads issue together
        int coff[NCH];
#pragma unroll
        for (int i = 0; i < NCH; i++) coff[i] = (64 * i < Kpad ? 64 * i : 0) + lane;
#pragma unroll 8
        for (int j = 0; j < d; j++) {
            float cv[NCH];
#pragma unroll
            for (int i = 0; i < NCH; i++) cv[i] = CT32[(size_t)j * Kpad + coff[i]];
#pragma unroll
            for (int r = 0; r < R; r++) {
                const float xj = (float)xs[wave][r][j];
#pragma unroll
                for (int i = 0; i < NCH; i++) acc[r][i] = fmaf(xj, cv[i], acc[r][i]);
            }
        }
        // per row: bound, U = min (s~ + e), candidate masks (wave-uniform)
        unsigned long long cm[R][NCH];
        int ncand[R];
        bool pr[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            // |x|^2 in fp64 over the lanes' f32 partials, rounded up (as the f32 path)
            double xn2 = (double)xn2p[r];
            for (int off = 32; off >= 1; off >>= 1) xn2 += __shfl_xor(xn2, off);
            xn2 = xn2 * (sizeof(TX) == 4 ? 1.0 + 0x1p-20 : 1.0 + 0x1p-19) + (sizeof(TX) == 4 ? 0.0 : 0x1p-280);
            const float nx = (float)(sqrt(xn2) * (1.0 + 0x1p-30));
            const float ex = (float)(0x1p-40 * xn2 * (1.0 + 0x1p-18) + 1e-30);
            float lo[NCH];
            float U = __builtin_inff();
            bool finite = nx <= 3.0e38f;
#pragma unroll
            for (int i = 0; i < NCH; i++) {
                const int c = lane + 64 * i;
                lo[i] = __builtin_inff();
                if (c < K) {
                    const float E = fmaf(nx, chunkc[2 * i], chunkc[2 * i + 1] + ex);
                    const float sc = MET == 1 ? cconst[c] - acc[r][i] : fmaf(-2.f, acc[r][i], cconst[c]);
                    lo[i] = sc - E;
                    const float hi = sc + E;
                    finite = finite && (hi - lo[i]) <= 3.0e38f;   // false for inf / nan
                    U = fminf(U, hi);
                }
            }
            for (int off = 32; off >= 1; off >>= 1) U = fminf(U, __shfl_xor(U, off));
            ncand[r] = 0;
#pragma unroll
            for (int i = 0; i < NCH; i++) {
                cm[r][i] = __ballot(lo[i] <= U);
                ncand[r] += __popcll(cm[r][i]);
            }
            pr[r] = r < nr && __all(finite) && ncand[r] >= 1;
        }
        // rows with <= RL candidates: lane RL r + k evaluates row r's k-th candidate
        {
            const int r = lane / RL, k = lane % RL;
            int c = -1;
            int seen = 0;
#pragma unroll
            for (int rr = 0; rr < R; rr++) {
                if (rr != r || !pr[rr] || ncand[rr] > RL) continue;
#pragma unroll
                for (int i = 0; i < NCH; i++) {
                    const int n = __popcll(cm[rr][i]);
                    if (c < 0 && k >= seen && k < seen + n) {
                        unsigned long long m = cm[rr][i];
                        for (int t = k - seen; t > 0; t--) m &= m - 1;
                        c = 64 * i + __builtin_ctzll(m);
                    }
                    seen += n;
                }
            }
            double best = 0.0;
            int bi = -1;
            if constexpr (MET == 0) {
                pruned_pick_euclid<RL>(xs[wave][r], C, d, c, exact_dist != 0, best, bi);   // within the row's lanes
            } else {
                if (c >= 0) {
                    best = pruned_dist<MET>(xs[wave][r], C + (size_t)c * d, d);
                    bi = c;
                }
                group_argmin<RL>(best, bi);
            }
            if (k == 0 && bi >= 0) {
                assign[myrow[r]] = bi;
                dist[myrow[r]] = best;
            }
        }
        // the other rows, one at a time with the whole wave
        for (int r = 0; r < nr; r++) {
            if (pr[r] && ncand[r] <= RL) continue;
            const bool prune = pr[r] && ncand[r] <= 64;
            const TX* xr = xs[wave][r];
            double best = 0.0;
            int bi = -1;
            if (prune) {
                // lane k takes the k-th candidate (increasing c)
                int c = -1, seen = 0;
#pragma unroll
                for (int i = 0; i < NCH; i++) {
                    const int n = __popcll(cm[r][i]);
                    if (c < 0 && lane >= seen && lane < seen + n) {
                        unsigned long long m = cm[r][i];
                        for (int t = lane - seen; t > 0; t--) m &= m - 1;
                        c = 64 * i + __builtin_ctzll(m);
                    }
                    seen += n;
                }
                if constexpr (MET == 0) {
                    pruned_pick_euclid<64>(xr, C, d, c, exact_dist != 0, best, bi);
                } else if (c >= 0) {
                    best = pruned_dist<MET>(xr, C + (size_t)c * d, d);
                    bi = c;
                }
            } else {
                for (int c = lane; c < K; c += 64) {
                    const double dd = pruned_dist<MET>(xr, C + (size_t)c * d, d);
                    // assignment.hpp:66: the -1 sentinel takes centroid 0's distance
                    // even if NaN, which then blocks every later '<'
                    if (bi < 0 ? (dd == dd || c == 0) : dd < best) { best = dd; bi = c; }
                }
            }
            for (int off = 32; off >= 1; off >>= 1) {
                const double ob = __shfl_xor(best, off);
                const int oi = __shfl_xor(bi, off);
                const bool take = oi >= 0 && (bi < 0 || ob < best || (ob == best && oi < bi));
                if (take) { best = ob; bi = oi; }
            }
            if (lane == 0) {
                assign[myrow[r]] = bi < 0 ? 0 : bi;
                dist[myrow[r]] = bi < 0 ? -1.0 : best;
            }
        }
        wave_sync();
    }
}

// 256 < K <= 1024: XPW_R rows per wave -- the centroid columns stream from L2
// once per XPW_R rows (at 2 rows per wave the C5 pass read ~36 GB of L2 for
// 140K listed rows) -- and the candidates of each row selected and evaluated in
// turn by the whole wave (per-row masks only: no [rows][chunks] mask array).
#ifndef XPW_ROWS
#define XPW_ROWS 4       // C5 whole call: 2 rows per wave (segmented) 5.46-5.51 ms; flat 2 / 4 / 8: 4.97 / 4.82-4.91 / 4.95-5.08
#endif
constexpr int XPW_MAXSEG = 4096;
template <typename TX, int MET = 0, int NCH = 16, int R = XPW_ROWS>
__global__ __launch_bounds__(64 * XP_WAVES) void assign_pruned_wide_kernel(
    const TX* __restrict__ X, int d, const double* __restrict__ C, const float* __restrict__ CT32,
    const float* __restrict__ cconst, int K, int Kpad, const int32_t* __restrict__ rows,
    const unsigned long long* __restrict__ row_count, int64_t max_rows, int32_t* __restrict__ assign,
    double* __restrict__ dist, const int32_t* __restrict__ seg_counts, int64_t seg_rows, int nseg, int exact_dist) {
    __shared__ TX xs[XP_WAVES][R][XB_DMAX];
    __shared__ int gpre[XPW_MAXSEG + 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // segmented lists (one per fused block): the groups of every segment in one
    // flat index space, so the waves share the work whatever the segments' sizes
    // (per-segment waves left the pass waiting on the fullest segments)
    int64_t ngroups;
    if (seg_counts) {
        for (int sg = threadIdx.x; sg < nseg; sg += 64 * XP_WAVES) gpre[sg + 1] = (seg_counts[2 * sg] + R - 1) / R;
        __syncthreads();
        if (threadIdx.x == 0) {
            gpre[0] = 0;
            for (int sg = 0; sg < nseg; sg++) gpre[sg + 1] += gpre[sg];
        }
        __syncthreads();
        ngroups = gpre[nseg];
    } else {
        int64_t total = (int64_t)*row_count;
        if (total > max_rows) total = max_rows;
        ngroups = (total + R - 1) / R;
    }
    const float* chunkc = cconst + Kpad;
    const int64_t g0 = (int64_t)blockIdx.x * XP_WAVES + wave, gstride = (int64_t)gridDim.x * XP_WAVES;
    for (int64_t g = g0; g < ngroups; g += gstride) {
        const int32_t* grows;
        int64_t gbase, cnt;
        if (seg_counts) {
            int lo = 0, hi = nseg;                  // gpre[lo] <= g < gpre[hi]
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (gpre[mid] <= g) lo = mid; else hi = mid;
            }
            grows = rows + (int64_t)lo * seg_rows;
            gbase = (g - gpre[lo]) * R;
            cnt = seg_counts[2 * lo];
        } else {
            grows = rows;
            gbase = g * R;
            cnt = min((int64_t)*row_count, max_rows);
        }
        const int nr = (int)min((int64_t)R, cnt - gbase);
        int32_t myrow[R];
#pragma unroll
        for (int r = 0; r < R; r++) myrow[r] = grows[gbase + min(r, nr - 1)];   // pad with the last row
        float xn2p[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            TX xv[XB_DMAX / 64];
#pragma unroll
            for (int u = 0; u < XB_DMAX / 64; u++) {
                const int j = lane + 64 * u;
                xv[u] = j < d ? X[(int64_t)myrow[r] * d + j] : TX(0);
            }
            float q = 0.f;
#pragma unroll
            for (int u = 0; u < XB_DMAX / 64; u++) {
                const int j = lane + 64 * u;
                if (j < d) {
                    xs[wave][r][j] = xv[u];
                    q = fmaf((float)xv[u], (float)xv[u], q);
                }
            }
            xn2p[r] = q;
        }
        wave_sync();
        float acc[R][NCH];
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int i = 0; i < NCH; i++) acc[r][i] = 0.f;
        int coff[NCH];
#pragma unroll
        for (int i = 0; i < NCH; i++) coff[i] = (64 * i < Kpad ? 64 * i : 0) + lane;
#pragma unroll 2
        for (int j = 0; j < d; j++) {
            float cv[NCH];
#pragma unroll
            for (int i = 0; i < NCH; i++) cv[i] = CT32[(size_t)j * Kpad + coff[i]];
#pragma unroll
            for (int r = 0; r < R; r++) {
                const float xj = (float)xs[wave][r][j];
#pragma unroll
                for (int i = 0; i < NCH; i++) acc[r][i] = fmaf(xj, cv[i], acc[r][i]);
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (r >= nr) break;                     // wave-uniform
            double xn2 = (double)xn2p[r];
            for (int off = 32; off >= 1; off >>= 1) xn2 += __shfl_xor(xn2, off);
            xn2 = xn2 * (sizeof(TX) == 4 ? 1.0 + 0x1p-20 : 1.0 + 0x1p-19) + (sizeof(TX) == 4 ? 0.0 : 0x1p-280);
            const float nx = (float)(sqrt(xn2) * (1.0 + 0x1p-30));
            const float ex = (float)(0x1p-40 * xn2 * (1.0 + 0x1p-18) + 1e-30);
            float lo[NCH];
            float U = __builtin_inff();
            bool finite = nx <= 3.0e38f;
#pragma unroll
            for (int i = 0; i < NCH; i++) {
                const int c = lane + 64 * i;
                lo[i] = __builtin_inff();
                if (c < K) {
                    const float E = fmaf(nx, chunkc[2 * i], chunkc[2 * i + 1] + ex);
                    const float sc = MET == 1 ? cconst[c] - acc[r][i] : fmaf(-2.f, acc[r][i], cconst[c]);
                    lo[i] = sc - E;
                    const float hi = sc + E;
                    finite = finite && (hi - lo[i]) <= 3.0e38f;   // false for inf / nan
                    U = fminf(U, hi);
                }
            }
            for (int off = 32; off >= 1; off >>= 1) U = fminf(U, __shfl_xor(U, off));
            unsigned long long cm[NCH];
            int ncand = 0;
#pragma unroll
            for (int i = 0; i < NCH; i++) {
                cm[i] = __ballot(lo[i] <= U);
                ncand += __popcll(cm[i]);
            }
            const bool prune = __all(finite) && ncand >= 1 && ncand <= 64;
            const TX* xr = xs[wave][r];
            double best = 0.0;
            int bi = -1;
            if (prune) {
                // lane k takes the k-th candidate (increasing c)
                int c = -1, seen = 0;
#pragma unroll
                for (int i = 0; i < NCH; i++) {
                    const int n = __popcll(cm[i]);
                    if (c < 0 && lane >= seen && lane < seen + n) {
                        unsigned long long m = cm[i];
                        for (int t = lane - seen; t > 0; t--) m &= m - 1;
                        c = 64 * i + __builtin_ctzll(m);
                    }
                    seen += n;
                }
                if constexpr (MET == 0) {
                    pruned_pick_euclid<64>(xr, C, d, c, exact_dist != 0, best, bi);
                } else if (c >= 0) {
                    best = pruned_dist<MET>(xr, C + (size_t)c * d, d);
                    bi = c;
                }
            } else {
                for (int c = lane; c < K; c += 64) {
                    const double dd = pruned_dist<MET>(xr, C + (size_t)c * d, d);
                    // assignment.hpp:66: the -1 sentinel takes centroid 0's distance
                    // even if NaN, which then blocks every later '<'
                    if (bi < 0 ? (dd == dd || c == 0) : dd < best) { best = dd; bi = c; }
                }
            }
            for (int off = 32; off >= 1; off >>= 1) {
                const double ob = __shfl_xor(best, off);
                const int oi = __shfl_xor(bi, off);
                const bool take = oi >= 0 && (bi < 0 || ob < best || (ob == best && oi < bi));
                if (take) { best = ob; bi = oi; }
            }
            if (lane == 0) {
                assign[myrow[r]] = bi < 0 ? 0 : bi;
                dist[myrow[r]] = bi < 0 ? -1.0 : best;
            }
        }
        wave_sync();
    }
}

int launch_assign_pruned_prep(hipStream_t s, bool xf64, int d, const double* C, int K, float* ws, int metric) {
    if (d > XB_DMAX || K > 1024) {
        set_error("launch_assign_pruned_prep: unsupported shape");
        return -1;
    }
    const int Kpad = (K + 63) / 64 * 64;
    float* cconst = ws + (size_t)d * Kpad;
    if (hipMemsetAsync(cconst + Kpad, 0, (size_t)(Kpad / 64) * 2 * 4, s) != hipSuccess) return kstatus("pruned prep");
    hipLaunchKernelGGL(exact_prep_kernel, dim3((unsigned)Kpad), dim3(64), 0, s, C, K, Kpad, d, xf64 ? 1 : 0, ws, cconst,
                       metric);
    return kstatus("exact_prep_kernel");
}

int launch_assign_pruned_list(hipStream_t s, Pts X, int d, const double* C, int K, float* ws,
                              const int32_t* rows, const unsigned long long* row_count, int64_t max_rows,
                              int32_t* assign, double* dist, const int32_t* seg_counts, int64_t seg_rows, int nseg,
                              int metric, int exact_dist, bool prepped) {
    if (max_rows <= 0) return 0;
    if (d > XB_DMAX || K > 1024 || (seg_counts && nseg <= 0)) {
        set_error("launch_assign_pruned_list: unsupported shape");
        return -1;
    }
    const int Kpad = (K + 63) / 64 * 64;
    float* CT32 = ws;
    float* cconst = ws + (size_t)d * Kpad;
    if (!prepped) {
        int rc = launch_assign_pruned_prep(s, X.f64, d, C, K, ws, metric);
        if (rc) return rc;
    }
    // K <= 256: 8 rows per wave over 4 chunks; K <= 1024: 2 rows per wave over 16
    const bool wide = Kpad > 256;
    const bool flat = wide && (!seg_counts || nseg <= XPW_MAXSEG);
    const int R = wide ? (flat ? XPW_ROWS : XP_WR) : XP_R;     // groups of R rows
    const int64_t groups = (max_rows + R - 1) / R;
    const int64_t blocks = seg_counts ? (int64_t)nseg * XP_SPLIT : std::min<int64_t>((groups + XP_WAVES - 1) / XP_WAVES, 2048);
#define XP_LAUNCH(TX, NCH, RR, MT, XP)                                                                              \
    hipLaunchKernelGGL((assign_pruned_kernel<TX, NCH, RR, MT>), dim3((unsigned)blocks), dim3(64 * XP_WAVES), 0, s, XP, \
                       d, C, CT32, cconst, K, Kpad, rows, row_count, max_rows, assign, dist, seg_counts, seg_rows, exact_dist)
#define XPW_LAUNCH(TX, MT, NC, RW, XP)                                                                           \
    hipLaunchKernelGGL((assign_pruned_wide_kernel<TX, MT, NC, RW>), dim3((unsigned)wblocks), dim3(64 * XP_WAVES), 0, s, \
                       XP, d, C, CT32, cconst, K, Kpad, rows, row_count, max_rows, assign, dist, seg_counts, seg_rows, nseg, \
                       exact_dist)
    const int64_t wblocks = std::min<int64_t>((groups + XP_WAVES - 1) / XP_WAVES, 1024);
    if (flat) {
        if (metric == 1) {
            if (X.f64) XPW_LAUNCH(double, 1, 16, XPW_ROWS, X.d()); else XPW_LAUNCH(float, 1, 16, XPW_ROWS, X.f());
        } else {
            if (X.f64) XPW_LAUNCH(double, 0, 16, XPW_ROWS, X.d()); else XPW_LAUNCH(float, 0, 16, XPW_ROWS, X.f());
        }
    } else if (metric == 1) {
        if (X.f64) {
            if (wide) XP_LAUNCH(double, 16, XP_WR, 1, X.d()); else XP_LAUNCH(double, 4, XP_R, 1, X.d());
        } else {
            if (wide) XP_LAUNCH(float, 16, XP_WR, 1, X.f()); else XP_LAUNCH(float, 4, XP_R, 1, X.f());
        }
    } else if (X.f64) {
        if (wide) XP_LAUNCH(double, 16, XP_WR, 0, X.d()); else XP_LAUNCH(double, 4, XP_R, 0, X.d());
    } else {
        if (wide) XP_LAUNCH(float, 16, XP_WR, 0, X.f()); else XP_LAUNCH(float, 4, XP_R, 0, X.f());
    }
#undef XP_LAUNCH
#undef XPW_LAUNCH
    return kstatus("assign_pruned_kernel");
}

int launch_assign_exact_list(hipStream_t s, Pts X, int d, const double* C, int K, double* CT,
                             const int32_t* rows, const unsigned long long* row_count, int64_t max_rows,
                             int32_t* assign, double* dist, const int32_t* seg_counts, int64_t seg_rows, int nseg) {
    if (max_rows <= 0) return 0;
    if (d > XB_DMAX || (seg_counts && nseg <= 0)) {
        set_error("launch_assign_exact_list: unsupported shape");
        return -1;
    }
    const int Kpad = (K + 255) / 256 * 256;     // CT row stride: whole 256-centroid passes, no bounds checks
    const int64_t ne = (int64_t)d * Kpad;
    hipLaunchKernelGGL(transpose_centroids_kernel, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, s, C, K, Kpad, d, CT);
    const int64_t groups = (max_rows + XB_R - 1) / XB_R;
    const int64_t blocks = seg_counts ? (int64_t)nseg * XB_SPLIT : std::min<int64_t>((groups + XB_WAVES - 1) / XB_WAVES, 2048);
    if (X.f64)
        hipLaunchKernelGGL(assign_exact_batch_kernel<double>, dim3((unsigned)blocks), dim3(64 * XB_WAVES), 0, s, X.d(),
                           d, CT, K, Kpad, rows, row_count, max_rows, assign, dist, seg_counts, seg_rows);
    else
        hipLaunchKernelGGL(assign_exact_batch_kernel<float>, dim3((unsigned)blocks), dim3(64 * XB_WAVES), 0, s, X.f(),
                           d, CT, K, Kpad, rows, row_count, max_rows, assign, dist, seg_counts, seg_rows);
    return kstatus("assign_exact_batch_kernel");
}

// Centroid override (assignment.hpp:77-78): in c order, so the last centroid
// that points at a row wins.
__global__ void assign_override_kernel(const int32_t* __restrict__ src, int K, int64_t N,
                                       int32_t* __restrict__ assign, double* __restrict__ dist) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= K) return;
    const int32_t r = src[c];
    if (r < 0 || r >= N) return;
    for (int c2 = c + 1; c2 < K; c2++)      // a later centroid on the same row wins
        if (src[c2] == r) return;
    assign[r] = c;
    dist[r] = 0.0;
}

// Same, one block with the K source rows in LDS (K <= OV_LDS_MAX): thread c
// scans the later entries 4 at a time (ds_read_b128, 4 independent reads in
// flight) instead of K^2/2 dependent global loads.
constexpr int OV_LDS_MAX = 8192;
__global__ __launch_bounds__(1024) void assign_override_lds_kernel(const int32_t* __restrict__ src, int K, int64_t N,
                                                                  int32_t* __restrict__ assign,
                                                                  double* __restrict__ dist) {
    __shared__ __attribute__((aligned(16))) int32_t ls[OV_LDS_MAX + 16];
    const int Kp = (K + 15) & ~15;
    for (int c = threadIdx.x; c < Kp + 16; c += blockDim.x) ls[c] = c < K ? src[c] : -1;
    __syncthreads();
    for (int c = threadIdx.x; c < K; c += blockDim.x) {
        const int32_t r = ls[c];
        if (r < 0 || r >= N) continue;
        bool later = false;
        for (int b = (c + 1) & ~15; b < Kp && !later; b += 16) {
            const int4 v0 = *reinterpret_cast<const int4*>(ls + b);
            const int4 v1 = *reinterpret_cast<const int4*>(ls + b + 4);
            const int4 v2 = *reinterpret_cast<const int4*>(ls + b + 8);
            const int4 v3 = *reinterpret_cast<const int4*>(ls + b + 12);
            const int w[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                               v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
#pragma unroll
            for (int t = 0; t < 16; t++) later |= b + t > c && w[t] == r;
        }
        if (!later) {                     // a later centroid on the same row wins
            assign[r] = c;
            dist[r] = 0.0;
        }
    }
}

int launch_assign_override(hipStream_t s, const int32_t* src_rows, int K, int64_t N, int32_t* assign,
                           double* dist) {
    if (K <= OV_LDS_MAX)
        hipLaunchKernelGGL(assign_override_lds_kernel, dim3(1), dim3(1024), 0, s, src_rows, K, N, assign, dist);
    else
        hipLaunchKernelGGL(assign_override_kernel, dim3((K + 255) / 256), dim3(256), 0, s, src_rows, K, N, assign,
                           dist);
    return kstatus("assign.hip");
}

__global__ void add_counter_kernel(unsigned long long* dst, const unsigned long long* src) {
    if (threadIdx.x == 0) *dst += *src;
}

int launch_add_counter(hipStream_t s, unsigned long long* dst, const unsigned long long* src) {
    hipLaunchKernelGGL(add_counter_kernel, dim3(1), dim3(1), 0, s, dst, src);
    return kstatus("assign.hip");
}

// stats[dst_idx[i]] += src[i] for i < n (n <= 8): the per-call statistics in one launch
struct CounterAdds {
    int n;
    int dst[8];
    const unsigned long long* src[8];
};
__global__ void add_counters_kernel(unsigned long long* stats, CounterAdds c) {
    if ((int)threadIdx.x < c.n) atomicAdd(stats + c.dst[threadIdx.x], *c.src[threadIdx.x]);
}

int launch_add_counters(hipStream_t s, unsigned long long* stats, int n, const int* dst_idx,
                        const unsigned long long* const* src) {
    if (n <= 0) return 0;
    if (n > 8) {
        set_error("launch_add_counters: at most 8 counters");
        return -1;
    }
    CounterAdds c;
    c.n = n;
    for (int i = 0; i < n; i++) { c.dst[i] = dst_idx[i]; c.src[i] = src[i]; }
    hipLaunchKernelGGL(add_counters_kernel, dim3(1), dim3(64), 0, s, stats, c);
    return kstatus("assign.hip");
}

}  // namespace lshkm
