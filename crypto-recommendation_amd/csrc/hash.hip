// hash.hip — random-projection hash families on gfx950.
//
// Replaces, bit-exactly:
//   EuclideanHGen::generate   lib/generators/euclidean_h_gen.hpp:73-76
//   CustVector::inner_product lib/data_structures/cust_vector.hpp:105-121
//   EuclideanPhiGen::generate lib/generators/euclidean_phi_gen.hpp:77-92
//   CosineHGen / CosineGGen   lib/generators/cosine_h_gen.hpp:67-74, cosine_g_gen.hpp:58-66
//   HypercubeGen over CosineHGen lib/generators/hypercube_gen.hpp:63-73
//   insertVector's bucket index mod(generate(v), nb) lib/data_structures/cust_hashtable.hpp:68
//
// Layout: a block takes 64 points; the 64 rows are staged once into LDS
// (coalesced loads), then wave w of 4 computes a contiguous slice of the L*k
// projections for all 64 points, one point per lane. Projections are read as
// wave-uniform scalar loads from a transposed [d][LKpad] fp64 table, so each
// j step is one LDS read + one cvt + fpw fp64 FMAs per lane.
//
// Exactness: the reference sums double-rounded products in x87 long double.
// fp32 x fp32 products are exact in fp64, so the fp64 FMA chain differs from
// the long-double chain by at most (d+2) 2^-52 (|v|.|x| + |t|) / w (+ 2^-51 |y|
// for the final two roundings); a floor (or sign) that this bound cannot
// certify is recomputed in the same kernel with the soft-x87 emulation
// (softx87.h), bit for bit what the reference computes. Bytes per point:
// 4d read + 4(L k) tuples + 8 L phi/bucket written.
#include "common.h"
#include "kernels.h"
#include "softx87.h"
#include "lshkm_synth.h"

namespace lshkm {

constexpr int HASH_PB = 64;      // points per block
constexpr int HASH_THREADS = 256;
constexpr int HASH_FB = 8;       // projections accumulated per pass

template <int MODE>
__global__ __launch_bounds__(HASH_THREADS) void proj_hash_kernel(
    const float* __restrict__ X, int64_t N, HashParams p, int32_t* __restrict__ out_h,
    int32_t* __restrict__ out_phi, int32_t* __restrict__ out_bucket, unsigned long long* __restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int d = p.d, LK = p.LK, ds = d + 1;
    float* xs = reinterpret_cast<float*>(smem);               // [64][d+1]
    int32_t* hs = reinterpret_cast<int32_t*>(xs + HASH_PB * ds);  // [64][LK]

    const int64_t p0 = (int64_t)blockIdx.x * HASH_PB;
    const int npts = (int)min((int64_t)HASH_PB, N - p0);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;

    // Stage rows: wave-strided rows, lane-strided columns (coalesced 256 B per instruction).
    const float* src = X + p0 * d;
    for (int pp = wave; pp < npts; pp += 4)
        for (int j = lane; j < d; j += 64) xs[pp * ds + j] = src[(int64_t)pp * d + j];
    __syncthreads();

    const int fpw = (LK + 3) / 4;
    const int f_begin = wave * fpw;
    const int f_end = min(f_begin + fpw, LK);
    const bool valid = lane < npts;
    const float* xr = xs + (valid ? lane : 0) * ds;

    for (int fb = f_begin; fb < f_end; fb += HASH_FB) {
        double acc[HASH_FB];
#pragma unroll
        for (int u = 0; u < HASH_FB; u++) acc[u] = 0.0;
        double xn2 = 0.0;
        const int cnt = min(HASH_FB, f_end - fb);
        for (int j = 0; j < d; j++) {
            const double xj = (double)xr[j];
            xn2 = fma(xj, xj, xn2);
            const double* prow = p.PT + (size_t)j * p.LKpad + fb;
#pragma unroll
            for (int u = 0; u < HASH_FB; u++)
                if (u < cnt) acc[u] = fma(prow[u], xj, acc[u]);
        }
        const double xn = sqrt(xn2) * (1.0 + 0x1p-40);
#pragma unroll
        for (int u = 0; u < HASH_FB; u++) {
            if (u >= cnt) continue;
            const int f = fb + u;
            const double P = p.pnorm[f] * xn;
            int32_t hv;
            if (MODE == HM_LSH_EUCLID || MODE == HM_CUBE_EUCLID_H) {
                const double tt = (double)p.t[f], ww = (double)p.w;
                const double y = (acc[u] + tt) / ww;
                const double B = ((double)(d + 2) * 0x1p-52 * (P + fabs(tt))) / ww + fabs(y) * 0x1p-51;
                const double lo = floor(y - B), hi = floor(y + B);
                if (lo == hi) {
                    hv = (int32_t)lo;
                } else {
                    // Exact: sequential x87 semantics (cust_vector.hpp:117-118, euclidean_h_gen.hpp:75).
                    sx80 s = sx_zero();
                    for (int j = 0; j < d; j++)
                        s = sx_add_double(s, __dmul_rn(p.PT[(size_t)j * p.LKpad + f], (double)xr[j]));
                    s = sx_add_double(s, tt);
                    hv = (int32_t)sx_floor_i64(sx_div(s, sx_from_float(p.w)));
                    if (valid) atomicAdd(stats + STAT_HASH_EXACT, 1ull);
                }
            } else {
                const double B = (double)(d + 3) * 0x1p-52 * P;
                if (acc[u] > B) hv = 1;
                else if (acc[u] < -B) hv = 0;
                else {
                    sx80 s = sx_zero();
                    for (int j = 0; j < d; j++)
                        s = sx_add_double(s, __dmul_rn(p.PT[(size_t)j * p.LKpad + f], (double)xr[j]));
                    hv = sx_ge_zero(s) ? 1 : 0;
                    if (valid) atomicAdd(stats + STAT_HASH_EXACT, 1ull);
                }
            }
            if (valid) hs[lane * LK + f] = hv;
        }
    }
    __syncthreads();

    const int L = p.L, k = p.k;
    if (MODE == HM_LSH_EUCLID) {
        if (out_h)
            for (int e = threadIdx.x; e < npts * LK; e += HASH_THREADS) out_h[p0 * LK + e] = hs[e];
        const int64_t M = 2147483647;   // int(pow(2,32)-5) under g++ (euclidean_phi_gen.hpp:70)
        for (int q = threadIdx.x; q < npts * L; q += HASH_THREADS) {
            const int pp = q / L, l = q - pp * L;
            uint32_t hn = 0;
            for (int i = 0; i < k; i++) {
                const int hi = hs[pp * LK + l * k + i];
                const int64_t temp = (int64_t)(int32_t)((uint32_t)hi * (uint32_t)p.r[l * k + i]);  // int*int
                hn += (uint32_t)(int32_t)((temp % M + M) % M);       // mod(long, int)
            }
            const uint32_t phi = (hn % 2147483647u + 2147483647u) % 2147483647u;  // mod(unsigned, int)
            if (out_phi) out_phi[p0 * L + q] = (int32_t)phi;
            if (out_bucket) out_bucket[p0 * L + q] = (int32_t)((uint64_t)phi % (uint64_t)p.nb);
        }
    } else if (MODE == HM_LSH_COSINE) {
        for (int q = threadIdx.x; q < npts * L; q += HASH_THREADS) {
            const int pp = q / L, l = q - pp * L;
            int g = 0;
            for (int i = 0; i < k; i++) g = (g << 1) + hs[pp * LK + l * k + i];
            if (out_phi) out_phi[p0 * L + q] = g;
            if (out_bucket) out_bucket[p0 * L + q] = g;
        }
    } else if (MODE == HM_CUBE_EUCLID_H) {
        for (int e = threadIdx.x; e < npts * LK; e += HASH_THREADS) out_h[p0 * LK + e] = hs[e];
    } else {
        for (int pp = threadIdx.x; pp < npts; pp += HASH_THREADS) {
            int v = 0;
            for (int i = 0; i < k; i++) v = (v << 1) + hs[pp * LK + i];
            out_h[p0 + pp] = v;
        }
    }
}

int launch_proj_hash(hipStream_t s, int mode, const float* X, int64_t N, const HashParams& p,
                     int32_t* out_h, int32_t* out_phi, int32_t* out_bucket, unsigned long long* stats) {
    if (N <= 0) return 0;
    const size_t lds = (size_t)HASH_PB * (p.d + 1) * 4 + (size_t)HASH_PB * p.LK * 4;
    const dim3 grid((unsigned)((N + HASH_PB - 1) / HASH_PB)), block(HASH_THREADS);
    switch (mode) {
        case HM_LSH_EUCLID:
            hipLaunchKernelGGL(proj_hash_kernel<HM_LSH_EUCLID>, grid, block, lds, s, X, N, p, out_h, out_phi, out_bucket, stats);
            break;
        case HM_LSH_COSINE:
            hipLaunchKernelGGL(proj_hash_kernel<HM_LSH_COSINE>, grid, block, lds, s, X, N, p, out_h, out_phi, out_bucket, stats);
            break;
        case HM_CUBE_EUCLID_H:
            hipLaunchKernelGGL(proj_hash_kernel<HM_CUBE_EUCLID_H>, grid, block, lds, s, X, N, p, out_h, out_phi, out_bucket, stats);
            break;
        default:
            hipLaunchKernelGGL(proj_hash_kernel<HM_CUBE_COSINE>, grid, block, lds, s, X, N, p, out_h, out_phi, out_bucket, stats);
            break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ------------------------------------------------------------ synthetic data
__global__ void synth_kernel(uint64_t seed, int64_t row0, int64_t total, int d, float* X) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / d, c = e - r * d;
        X[e] = lshkm_synth_value(seed, (uint64_t)(row0 + r), (uint64_t)d, (uint64_t)c);
    }
}

int launch_synth(hipStream_t s, uint64_t seed, int64_t row0, int64_t rows, int d, float* X) {
    const int64_t total = rows * d;
    if (total <= 0) return 0;
    const int64_t blocks = min((total + 255) / 256, (int64_t)256 * 64);
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)blocks), dim3(256), 0, s, seed, row0, total, d, X);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace lshkm
