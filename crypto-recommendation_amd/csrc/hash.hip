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

constexpr int HASH_PB = 64;      // points per block (at most; fewer for long rows)
constexpr int HASH_THREADS = 256;
constexpr size_t HASH_LDS_MAX = 96 * 1024;

// Row staging: 16-B loads when the row length allows (float4 / double2).
__device__ inline void hash_ld4(const float* p, double (&o)[4]) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
__device__ inline void hash_ld4(const double* p, double (&o)[4]) {
    const double2 a = *reinterpret_cast<const double2*>(p), b = *reinterpret_cast<const double2*>(p + 2);
    o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
}
template <typename TX> __host__ __device__ constexpr int hash_vec() { return 16 / sizeof(TX); }

// LDS row stride (elements): d rounded up to 4, plus 4 floats / 2 doubles
// (16 B), so the lanes' 16-B reads of their rows spread over the banks.
template <typename TX> __host__ __device__ inline int hash_dstride(int d) {
    return (d + 3) / 4 * 4 + (int)(16 / sizeof(TX));
}

// Per wave: FB projections (a contiguous, zero-padded column block of PT)
// accumulated together; PT is __restrict__ const so its wave-uniform reads
// become scalar (SMEM) loads that feed v_fma_f64 directly.
// TX = float: products v_j x_j are exact in fp64. TX = double: the reference
// rounds each product to double (SSE) before the x87 add; the FMA chain keeps
// them exact, so the two differ by the products' roundings (<= 2^-53 |v_j x_j|
// each) plus both chains' roundings: (d + 2) 2^-53 sum|v_j x_j| <= the
// (d + 2) 2^-52 |v||x| already charged, plus d 2^-1075 for subnormal products.
template <int MODE, int FB, typename TX>
__global__ __launch_bounds__(HASH_THREADS) void proj_hash_kernel(
    const TX* __restrict__ X, int64_t N, const double* __restrict__ PT, const float* __restrict__ tvec,
    const double* __restrict__ pnorm, const int32_t* __restrict__ rvec, HashParams p, int pb,
    int32_t* __restrict__ out_h, int32_t* __restrict__ out_phi, int32_t* __restrict__ out_bucket,
    unsigned long long* __restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int d = p.d, LK = p.LK, LKpad = p.LKpad, ds = hash_dstride<TX>(d);
    TX* xs = reinterpret_cast<TX*>(smem);                             // [pb][ds]
    int32_t* hs = reinterpret_cast<int32_t*>(xs + pb * ds);           // [pb][LK]

    const int64_t p0 = (int64_t)blockIdx.x * pb;
    const int npts = (int)min((int64_t)pb, N - p0);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;

    // Stage the block's rows (contiguous in HBM) into padded LDS rows.
    const TX* src = X + p0 * d;
    constexpr int V = hash_vec<TX>();
    if (d % V == 0) {
        const int dv = d / V, totv = npts * dv;
        for (int e = threadIdx.x; e < totv; e += HASH_THREADS) {
            const int r = e / dv, c = (e - r * dv) * V;
            *reinterpret_cast<float4*>(xs + r * ds + c) = *reinterpret_cast<const float4*>(src + (int64_t)e * V);
        }
    } else {
        for (int e = threadIdx.x; e < npts * d; e += HASH_THREADS) {
            const int r = e / d, c = e - r * d;
            xs[r * ds + c] = src[e];
        }
    }
    for (int e = threadIdx.x; e < pb * (ds - d); e += HASH_THREADS) {   // zero the pad columns
        const int r = e / (ds - d), c = d + (e - r * (ds - d));
        xs[r * ds + c] = (TX)0;
    }
    __syncthreads();

    const bool valid = lane < npts;
    const TX* xr = xs + (lane < pb ? lane : 0) * ds;
    const int chunks = LKpad / (4 * FB);
    const int d4 = (d + 3) >> 2;

    for (int ch = 0; ch < chunks; ch++) {
        const int fb = (wave * chunks + ch) * FB;
        if (fb >= LK) break;
        double acc[FB];
#pragma unroll
        for (int u = 0; u < FB; u++) acc[u] = 0.0;
        double xn2 = 0.0;
        // Constant address space: uniform reads here must become SMEM loads.
        const __attribute__((address_space(4))) double* prow =
            (const __attribute__((address_space(4))) double*)(PT + fb);
        for (int j4 = 0; j4 < d4; j4++) {
            double xa[4];
            hash_ld4(xr + 4 * j4, xa);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const double xj = xa[q];
                xn2 = fma(xj, xj, xn2);
#pragma unroll
                for (int u = 0; u < FB; u++) acc[u] = fma(prow[u], xj, acc[u]);   // pad rows/cols are 0
                prow += LKpad;
            }
        }
        const double xn = sqrt(xn2) * (1.0 + 0x1p-40);
#pragma unroll
        for (int u = 0; u < FB; u++) {
            const int f = fb + u;
            if (f >= LK) break;
            const double P = pnorm[f] * xn;
            int32_t hv;
            if (MODE == HM_LSH_EUCLID || MODE == HM_CUBE_EUCLID_H) {
                const double tt = (double)tvec[f], ww = (double)p.w;
                const double y = (acc[u] + tt) / ww;
                const double B = ((double)(d + 2) * 0x1p-52 * (P + fabs(tt)) + 0x1p-1000) / ww + fabs(y) * 0x1p-51;
                const double lo = floor(y - B), hi = floor(y + B);
                // certified, and inside the int range (the reference's FISTP stores
                // INT_MIN outside it); inf / nan never pass
                if (lo == hi && fabs(lo) < 0x1p31) {
                    hv = (int32_t)lo;
                } else {
                    // Exact: sequential x87 semantics (cust_vector.hpp:117-118, euclidean_h_gen.hpp:75).
                    SxSum s;
                    s.init();
                    for (int j = 0; j < d; j++) s.add(__dmul_rn(PT[(size_t)j * LKpad + f], (double)xr[j]));
                    hv = sx_hash_floor(s, tt, p.w);
                    if (valid) atomicAdd(stats + STAT_HASH_EXACT, 1ull);
                }
            } else {
                const double B = (double)(d + 3) * 0x1p-52 * P + 0x1p-1000;
                if (acc[u] > B && acc[u] < 0x1p1000) hv = 1;       // finite: no product overflowed
                else if (acc[u] < -B && acc[u] > -0x1p1000) hv = 0;
                else {
                    SxSum s;
                    s.init();
                    for (int j = 0; j < d; j++) s.add(__dmul_rn(PT[(size_t)j * LKpad + f], (double)xr[j]));
                    hv = sx_hash_sign(s);
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
                const int64_t temp = (int64_t)(int32_t)((uint32_t)hi * (uint32_t)rvec[l * k + i]);  // int*int
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

int hash_fb(int LK) {
    const int fpw = (LK + 3) / 4;
    return fpw <= 2 ? 2 : fpw <= 4 ? 4 : fpw <= 6 ? 6 : 8;
}

int hash_lkpad(int LK) {
    const int fb = hash_fb(LK), fpw = (LK + 3) / 4;
    return 4 * ((fpw + fb - 1) / fb) * fb;
}

template <int MODE, typename TX>
static void launch_mode(hipStream_t s, const TX* X, int64_t N, const HashParams& p, int32_t* out_h, int32_t* out_phi,
                        int32_t* out_bucket, unsigned long long* stats) {
    // points per block: 64 unless the staged rows would crowd the CU's LDS
    int pb = HASH_PB;
    auto lds_of = [&](int b) { return (size_t)b * hash_dstride<TX>(p.d) * sizeof(TX) + (size_t)b * p.LK * 4; };
    while (pb > 8 && lds_of(pb) > HASH_LDS_MAX) pb >>= 1;
    const dim3 grid((unsigned)((N + pb - 1) / pb)), block(HASH_THREADS);
    switch (hash_fb(p.LK)) {
#define HF_CASE(FB) case FB: hipLaunchKernelGGL((proj_hash_kernel<MODE, FB, TX>), grid, block, lds_of(pb), s, X, N, p.PT, \
                                              p.t, p.pnorm, p.r, p, pb, out_h, out_phi, out_bucket, stats); break;
        HF_CASE(2) HF_CASE(4) HF_CASE(6) HF_CASE(8)
#undef HF_CASE
    }
}

template <typename TX>
static void launch_tx(hipStream_t s, int mode, const TX* X, int64_t N, const HashParams& p, int32_t* out_h,
                      int32_t* out_phi, int32_t* out_bucket, unsigned long long* stats) {
    switch (mode) {
        case HM_LSH_EUCLID: launch_mode<HM_LSH_EUCLID>(s, X, N, p, out_h, out_phi, out_bucket, stats); break;
        case HM_LSH_COSINE: launch_mode<HM_LSH_COSINE>(s, X, N, p, out_h, out_phi, out_bucket, stats); break;
        case HM_CUBE_EUCLID_H: launch_mode<HM_CUBE_EUCLID_H>(s, X, N, p, out_h, out_phi, out_bucket, stats); break;
        default: launch_mode<HM_CUBE_COSINE>(s, X, N, p, out_h, out_phi, out_bucket, stats); break;
    }
}

int launch_proj_hash(hipStream_t s, int mode, Pts X, int64_t N, const HashParams& p,
                     int32_t* out_h, int32_t* out_phi, int32_t* out_bucket, unsigned long long* stats) {
    if (N <= 0) return 0;
    if (X.f64) launch_tx(s, mode, X.d(), N, p, out_h, out_phi, out_bucket, stats);
    else launch_tx(s, mode, X.f(), N, p, out_h, out_phi, out_bucket, stats);
    return kstatus("hash.hip");
}

// ------------------------------------------------------------ synthetic data
template <bool NORMAL>
__global__ void synth_kernel(uint64_t seed, int64_t row0, int64_t total, int d, float* X) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / d, c = e - r * d;
        X[e] = NORMAL ? lshkm_synth_normal_value(seed, (uint64_t)(row0 + r), (uint64_t)d, (uint64_t)c)
                      : lshkm_synth_value(seed, (uint64_t)(row0 + r), (uint64_t)d, (uint64_t)c);
    }
}

int launch_synth(hipStream_t s, uint64_t seed, int64_t row0, int64_t rows, int d, float* X, int kind) {
    const int64_t total = rows * d;
    if (total <= 0) return 0;
    const int64_t blocks = min((total + 255) / 256, (int64_t)256 * 64);
    if (kind == 1)
        hipLaunchKernelGGL(synth_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, seed, row0, total, d, X);
    else
        hipLaunchKernelGGL(synth_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, seed, row0, total, d, X);
    return kstatus("hash.hip");
}

}  // namespace lshkm
