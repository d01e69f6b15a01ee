// hash_mfma.hip — standalone random-projection hashing on split-f16 MFMA
// (fp32 points, d = 128, L*k <= 32): the build and query hashing of
// create_LSH_hashtables / create_hypercube and their queries
// (lib/lsh_cube.hpp:44-74, 77-106, 108-177) for all four families:
//   EuclideanHGen + EuclideanPhiGen (euclidean_h_gen.hpp:73-76,
//   euclidean_phi_gen.hpp:77-92): tuples, phi, bucket ID;
//   CosineHGen + CosineGGen (cosine_h_gen.hpp:67-76, cosine_g_gen.hpp:58-66);
//   EuclideanFGen's inner h values (euclidean_f_gen.hpp:65-79) and their range;
//   HypercubeGen over CosineHGen (hypercube_gen.hpp:63-73): the vertex.
//
// A wave takes 32 points as the MFMA B operand (lane half h: dims 16s+8h..+7
// of point lane&31) and the 32 projection rows (hi and lo f16 images, LDS) as
// A: per 16-dim step the lo products first, then the hi products, into one
// accumulator; the steps are added in f32. The certificate is the fused
// kernel's hash tile's (fused.hip): a floor (or a sign) is
// certified when the rigorous window |acc~ - the reference's x87 value| <=
// FU_A1H |v||x| + FU_A2 (sqrt(d)|x| + |v|_1) (+ the t and 1/w roundings) lies
// inside one integer cell (on one side of 0). The others — about 4% of rows
// at w = 0.4, fewer for larger w and for signs — are listed per block and
// redone by hash_mfma_fix_kernel from the exact row: the fp64 FMA chain with
// hash.hip's bound, and the soft-x87 emulation when that bound cannot decide.
// Bytes per point: 512 read + the outputs (LSH euclidean: 4 L k + 4 L).
#include "common.h"
#include "kernels.h"
#include "softx87.h"
#include "tile.h"

namespace lshkm {

constexpr int HMF_W = 4;        // waves per block
// blocks per CU: 2 (~160 VGPRs) so a wave's 16 row loads can all be in flight
// before its first MFMA (at 4 blocks the 128-VGPR cap made the scheduler issue
// them pair by pair next to each step: 8 serial trips per tile; C4 build 1.87
// -> 1.76 ms, C2 0.353 -> 0.337 ms)
constexpr int HMF_BPC = 2;
constexpr int HMF_VS = 33;      // per-wave value tile [32 points][33] int32
constexpr int hmf_lds_bytes() {
    return 2 * 32 * FU_RS * 2 + 4 * 32 * 4 + HMF_W * 32 * HMF_VS * 4 + 16;
}

struct HashMfmaArgs {
    const float* X;
    int64_t N;
    const _Float16* Vh;      // [>= 32][128] f16 hi of the projections (rows >= LK zero)
    const _Float16* Vl;      // lo
    const float* tv;         // [LK] (euclidean)
    const double* pnorm;     // [LK] |v|_2 rounded up
    const double* v1;        // [LK] |v|_1 rounded up
    const int32_t* rv;       // [LK] (LSH euclidean)
    const double* PT;        // [128][LKpad] fp64 projections (fix-up)
    float w;
    int L, k, LK, LKpad;
    BucketDiv bdiv;
    int32_t* out_h;          // LSH euclidean: tuples [N][LK]; cube euclidean: h [N][k]; cube cosine: vertex [N]
    int h16;                 // cube euclidean: h as int16 (saturated; the range in mm is the true one)
    int32_t* out_phi;        // LSH: [N][L] (may be null)
    int32_t* out_bucket;     // LSH: [N][L] (may be null)
    int32_t* mm;             // cube euclidean: [0] min h, [1] max h (atomics; pre-set by the caller)
    unsigned long long* list;    // per block: (row << 32) | mask of the uncertified functions
    int32_t* seg_counts;         // [grid]
    int64_t seg_rows;
    unsigned long long* stats;
};

// int16 h (cube euclidean): values outside the range saturate; the caller sees
// the true range in mm and hashes again as int32 then.
__device__ inline int16_t h_sat16(int32_t v) { return (int16_t)min(32767, max(-32768, v)); }

template <int MODE>
__global__ __launch_bounds__(64 * HMF_W, HMF_BPC) void hash_mfma_kernel(HashMfmaArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    _Float16* lvh = reinterpret_cast<_Float16*>(smem);
    _Float16* lvl = lvh + 32 * FU_RS;
    float* lP = reinterpret_cast<float*>(lvl + 32 * FU_RS);   // window coefficient of |x|
    float* lQ = lP + 32;                                       // constant window part
    float* lt = lQ + 32;
    int32_t* lr = reinterpret_cast<int32_t*>(lt + 32);
    int32_t* lval = lr + 32;                                   // [HMF_W][32][HMF_VS]
    int* lmisc = lval + HMF_W * 32 * HMF_VS;                   // [0] list count, [1] min, [2] max
    constexpr bool EUCLID = MODE == HM_LSH_EUCLID || MODE == HM_CUBE_EUCLID_H;

    for (int e = threadIdx.x; e < 32 * 16; e += 64 * HMF_W) {
        const int r = e >> 4, g = e & 15;
        *reinterpret_cast<float4*>(lvh + r * FU_RS + g * 8) = *reinterpret_cast<const float4*>(a.Vh + r * FU_D + g * 8);
        *reinterpret_cast<float4*>(lvl + r * FU_RS + g * 8) = *reinterpret_cast<const float4*>(a.Vl + r * FU_D + g * 8);
    }
    if (threadIdx.x < 32) {
        const int f = threadIdx.x;
        const bool on = f < a.LK;
        // euclidean: the window in units of y = (acc + t) / w (fused.hip's hash
        // tile); cosine: in units of the inner product itself
        const double iwu = EUCLID ? (double)(1.0f / a.w) * (1.0 + 0x1p-20) : 1.0;
        const double tf = EUCLID && on ? fabs((double)a.tv[f]) : 0.0;
        lP[f] = on ? (float)((FU_A1H * a.pnorm[f] * (1.0 + 0x1p-20) + FU_A2 * FU_SQRT_D) * iwu * (1.0 + 0x1p-18)) : 0.f;
        lQ[f] = on ? (float)((FU_A2 * a.v1[f] * (1.0 + 0x1p-20) + (0x1p-40 + 0x1p-23) * tf) * iwu * (1.0 + 0x1p-18) +
                             0x1p-126) : 0.f;
        lt[f] = on && EUCLID ? a.tv[f] : 0.f;
        lr[f] = on && MODE == HM_LSH_EUCLID ? a.rv[f] : 0;
    }
    if (threadIdx.x == 0) { lmisc[0] = 0; lmisc[1] = 0x7FFFFFFF; lmisc[2] = (int)0x80000000; }
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 31, h = lane >> 5;
    const int LK = a.LK, L = a.L, k = a.k;
    const int64_t ntiles = (a.N + 31) >> 5;
    int32_t* lv = lval + wave * 32 * HMF_VS;
    unsigned long long* seg = a.list + (int64_t)blockIdx.x * a.seg_rows;
    const float iw = EUCLID ? 1.0f / a.w : 1.f;
    constexpr float G = (0x1p-22f + 0x1p-20f) * (1.f + 0x1p-18f);
    int hmin = 0x7FFFFFFF, hmax = (int)0x80000000;
    const _Float16* vh_row = lvh + col * FU_RS + 8 * h;
    const _Float16* vl_row = lvl + col * FU_RS + 8 * h;

    for (int64_t tile = (int64_t)blockIdx.x * HMF_W + wave; tile < ntiles; tile += (int64_t)gridDim.x * HMF_W) {
        const int64_t row = tile * 32 + col;
        const bool valid = row < a.N;
        float xf[64];
        {
            const float* xr = a.X + (valid ? row : a.N - 1) * FU_D + 8 * h;
#pragma unroll
            for (int s = 0; s < 8; s++) {
                const float4 p0 = *reinterpret_cast<const float4*>(xr + 16 * s);
                const float4 p1 = *reinterpret_cast<const float4*>(xr + 16 * s + 4);
                xf[8 * s + 0] = p0.x; xf[8 * s + 1] = p0.y; xf[8 * s + 2] = p0.z; xf[8 * s + 3] = p0.w;
                xf[8 * s + 4] = p1.x; xf[8 * s + 5] = p1.y; xf[8 * s + 6] = p1.z; xf[8 * s + 7] = p1.w;
            }
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the 16 loads ahead of the MFMA steps
        float2v n2a = {0.f, 0.f}, n2b = {0.f, 0.f}, r2 = {0.f, 0.f};
        floatx16 tot;
#pragma unroll
        for (int s = 0; s < 8; s++) {
            half8 bh, bl;
            split8_hi<true>(xf + 8 * s, bh, bl, r2);
#pragma unroll
            for (int j = 0; j < 8; j += 4) {
                const float2v u = {xf[8 * s + j], xf[8 * s + j + 1]}, v = {xf[8 * s + j + 2], xf[8 * s + j + 3]};
                n2a = __builtin_elementwise_fma(u, u, n2a);
                n2b = __builtin_elementwise_fma(v, v, n2b);
            }
            const half8 ah = *reinterpret_cast<const half8*>(vh_row + 16 * s);
            const half8 al = *reinterpret_cast<const half8*>(vl_row + 16 * s);
            const floatx16 z = {};
            floatx16 acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, z, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
            if (s == 0) {
                tot = acc;
            } else {
#pragma unroll
                for (int r = 0; r < 16; r += 2) {
                    const float2v t2 = {tot[r], tot[r + 1]}, a2 = {acc[r], acc[r + 1]};
                    const float2v u2 = t2 + a2;
                    tot[r] = u2.x;
                    tot[r + 1] = u2.y;
                }
            }
        }
        float xn2f = (n2a.x + n2a.y) + (n2b.x + n2b.y);
        xn2f += __shfl_xor(xn2f, 32);
        const bool x_ok = xn2f <= FU_RANGE * FU_RANGE;          // false for inf / nan too
        // |x| rounded up: the f32 sum of squares inflated by 2^-16 (> d 2^-24)
        const float nxf = (float)(sqrt((double)xn2f * (1.0 + 0x1p-16)) * (1.0 + 0x1p-20));
        // value and certificate of function f = 8g + 4h + q (D register 4g + q)
        uint32_t fmask = 0;
        // LSH euclidean with k = 4 (the reference default): table l = 2g + h is
        // D registers 4g..4g+3 of lane half h, so tuples, phi and the bucket are
        // written from registers (fused.hip's layout)
        const bool k4 = MODE == HM_LSH_EUCLID && k == 4;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            int32_t hv4[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int f = 8 * g + 4 * h + q;
                hv4[q] = 0;
                if (f >= LK) continue;
                int32_t v;
                bool ok;
                if (EUCLID) {
                    const float y = (tot[4 * g + q] + lt[f]) * iw;
                    const float B = fmaf(fabsf(y), G, fmaf(nxf, lP[f], lQ[f]));
                    const float lo = floorf(y - B), hi = floorf(y + B);
                    v = (int32_t)lo;
                    ok = lo == hi;
                } else {
                    const float u = tot[4 * g + q];
                    const float B = fmaf(nxf, lP[f], lQ[f]);
                    v = u >= 0.f ? 1 : 0;
                    ok = fabsf(u) > B;
                }
                if (!(ok && x_ok)) fmask |= 1u << f;
                hv4[q] = v;
                if (!k4) lv[col * HMF_VS + f] = v;
                if (MODE == HM_CUBE_EUCLID_H && ok && x_ok && valid) {
                    hmin = min(hmin, v);
                    hmax = max(hmax, v);
                }
            }
            if (MODE == HM_LSH_EUCLID && k4) {
                const int l = 2 * g + h;
                if (l < L && valid) {
                    const int64_t o = row * L + l;
                    *reinterpret_cast<int4*>(a.out_h + o * 4) = make_int4(hv4[0], hv4[1], hv4[2], hv4[3]);
                    uint32_t hn = 0;
#pragma unroll
                    for (int q = 0; q < 4; q++) hn += phi_term(hv4[q], lr[4 * l + q]);
                    const uint32_t ph = phi_final(hn);
                    if (a.out_phi) a.out_phi[o] = (int32_t)ph;
                    if (a.out_bucket) a.out_bucket[o] = bucket_fast(ph, a.bdiv);
                }
            }
        }
        fmask |= __shfl_xor(fmask, 32);
        const unsigned long long fb = __ballot(valid && fmask != 0u && h == 1);
        if (fb) {
            const int leader = __builtin_ctzll(fb);
            int base = 0;
            if (lane == leader) base = atomicAdd(lmisc, __popcll(fb));
            base = __shfl(base, leader);
            if (valid && fmask != 0u && h == 1)
                seg[base + __popcll(fb & ((1ull << lane) - 1ull))] = ((unsigned long long)row << 32) | fmask;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // outputs, lanes over (point, value) pairs of the tile
        const int npts = (int)min((int64_t)32, a.N - tile * 32);
        const int64_t r0 = tile * 32;
        if ((MODE == HM_LSH_EUCLID && !k4) || MODE == HM_CUBE_EUCLID_H) {
            if (MODE == HM_CUBE_EUCLID_H && a.h16) {
                int16_t* o16 = reinterpret_cast<int16_t*>(a.out_h) + r0 * LK;
                for (int e = lane; e < npts * LK; e += 64) {
                    const int p = e / LK, f = e - p * LK;
                    o16[e] = h_sat16(lv[p * HMF_VS + f]);
                }
            } else if (a.out_h) {
                for (int e = lane; e < npts * LK; e += 64) {
                    const int p = e / LK, f = e - p * LK;
                    a.out_h[r0 * LK + e] = lv[p * HMF_VS + f];
                }
            }
        }
        if (MODE == HM_LSH_EUCLID && !k4) {
            for (int e = lane; e < npts * L; e += 64) {
                const int p = e / L, l = e - p * L;
                uint32_t hn = 0;
                for (int i = 0; i < k; i++) hn += phi_term(lv[p * HMF_VS + l * k + i], lr[l * k + i]);
                const uint32_t ph = phi_final(hn);
                if (a.out_phi) a.out_phi[r0 * L + e] = (int32_t)ph;
                if (a.out_bucket) a.out_bucket[r0 * L + e] = bucket_fast(ph, a.bdiv);
            }
        } else if (MODE == HM_LSH_COSINE) {
            for (int e = lane; e < npts * L; e += 64) {
                const int p = e / L, l = e - p * L;
                int gv = 0;
                for (int i = 0; i < k; i++) gv = (gv << 1) + lv[p * HMF_VS + l * k + i];
                if (a.out_phi) a.out_phi[r0 * L + e] = gv;
                if (a.out_bucket) a.out_bucket[r0 * L + e] = gv;
            }
        } else if (MODE == HM_CUBE_COSINE) {
            if (lane < npts) {
                int vtx = 0;
                for (int i = 0; i < k; i++) vtx = (vtx << 1) + lv[lane * HMF_VS + i];
                a.out_h[r0 + lane] = vtx;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (MODE == HM_CUBE_EUCLID_H) {
        for (int off = 32; off >= 1; off >>= 1) {
            hmin = min(hmin, __shfl_xor(hmin, off));
            hmax = max(hmax, __shfl_xor(hmax, off));
        }
        if (lane == 0) { atomicMin(lmisc + 1, hmin); atomicMax(lmisc + 2, hmax); }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a.seg_counts[blockIdx.x] = lmisc[0];
        if (MODE == HM_CUBE_EUCLID_H && lmisc[1] <= lmisc[2]) {
            atomicMin(a.mm, lmisc[1]);
            atomicMax(a.mm + 1, lmisc[2]);
        }
    }
}

// Exact value of function f for one fp32 row: hash.hip's fp64 FMA chain and
// bound (the row streamed in 32-dim chunks, the projections read through the
// cache), then the soft-x87 chain when that bound cannot decide.
template <bool EUCLID>
__device__ int32_t hmf_exact(const float* __restrict__ xrow, const double* __restrict__ pt, int LKpad, int f,
                             double tt, float w, double pn, unsigned long long* stats) {
    double acc = 0.0, xn2 = 0.0;
#pragma unroll 1
    for (int c = 0; c < FU_D; c += 32) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = *reinterpret_cast<const float4*>(xrow + c + 4 * u);
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const float xs[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const double xj = (double)xs[e];
                xn2 = fma(xj, xj, xn2);
                acc = fma(pt[(size_t)(c + 4 * u + e) * LKpad + f], xj, acc);
            }
        }
    }
    const double P = pn * sqrt(xn2) * (1.0 + 0x1p-40);
    if (EUCLID) {
        const double ww = (double)w;
        const double y = (acc + tt) / ww;
        const double B = ((double)(FU_D + 2) * 0x1p-52 * (P + fabs(tt)) + 0x1p-1000) / ww + fabs(y) * 0x1p-51;
        const double lo = floor(y - B), hi = floor(y + B);
        if (lo == hi && fabs(lo) < 0x1p31) return (int32_t)lo;
    } else {
        const double B = (double)(FU_D + 3) * 0x1p-52 * P + 0x1p-1000;
        if (acc > B && acc < 0x1p1000) return 1;
        if (acc < -B && acc > -0x1p1000) return 0;
    }
    SxSum s;
    s.init();
    for (int j = 0; j < FU_D; j++) s.add(__dmul_rn(pt[(size_t)j * LKpad + f], (double)xrow[j]));
    atomicAdd(stats + STAT_HASH_EXACT, 1ull);
    return EUCLID ? sx_hash_floor(s, tt, w) : sx_hash_sign(s);
}

constexpr int HMF_FIX_THREADS = 256;

// Lane = listed row: the flagged functions exactly, then the outputs that
// depend on them (LSH euclidean: the touched tables' phi / bucket from the
// stored tuples, whose other values are certified; cosine: the flagged bits
// of g / the vertex; cube euclidean: h and its range). One block per list
// segment; the fp64 projections are read through the cache (no LDS staging).
template <int MODE>
__global__ __launch_bounds__(HMF_FIX_THREADS) void hash_mfma_fix_kernel(HashMfmaArgs a) {
    constexpr bool EUCLID = MODE == HM_LSH_EUCLID || MODE == HM_CUBE_EUCLID_H;
    const int segi = blockIdx.x;
    const int n = a.seg_counts[segi];
    if (n == 0) return;                                 // block-uniform
    const int LK = a.LK, L = a.L, k = a.k;
    const double* __restrict__ pt = a.PT;
    const unsigned long long* list = a.list + (int64_t)segi * a.seg_rows;
    for (int e = threadIdx.x; e < n; e += HMF_FIX_THREADS) {
        const unsigned long long ent = list[e];
        const int64_t row = (int64_t)(ent >> 32);
        const uint32_t mask = (uint32_t)ent;
        const float* xrow = a.X + row * FU_D;
        uint32_t bits = 0;
        for (uint32_t m = mask; m; m &= m - 1) {
            const int f = __builtin_ctz(m);
            const int32_t v = hmf_exact<EUCLID>(xrow, pt, a.LKpad, f, EUCLID ? (double)a.tv[f] : 0.0, a.w,
                                                a.pnorm[f], a.stats);
            if (MODE == HM_LSH_EUCLID || MODE == HM_CUBE_EUCLID_H) {
                if (MODE == HM_CUBE_EUCLID_H && a.h16)
                    reinterpret_cast<int16_t*>(a.out_h)[row * LK + f] = h_sat16(v);
                else if (a.out_h)
                    a.out_h[row * LK + f] = v;
                if (MODE == HM_CUBE_EUCLID_H) { atomicMin(a.mm, v); atomicMax(a.mm + 1, v); }
            }
            bits |= (uint32_t)v << f;
        }
        if (MODE == HM_LSH_EUCLID) {
            const uint32_t kmask = k >= 32 ? 0xFFFFFFFFu : ((1u << k) - 1u);
            for (int l = 0; l < L; l++) {
                if (!(mask & (kmask << (l * k)))) continue;
                uint32_t hn = 0;
                for (int i = 0; i < k; i++) hn += phi_term(a.out_h[row * LK + l * k + i], a.rv[l * k + i]);
                const uint32_t ph = phi_final(hn);
                if (a.out_phi) a.out_phi[row * L + l] = (int32_t)ph;
                if (a.out_bucket) a.out_bucket[row * L + l] = bucket_fast(ph, a.bdiv);
            }
        } else if (MODE == HM_LSH_COSINE) {
            const uint32_t kmask = k >= 32 ? 0xFFFFFFFFu : ((1u << k) - 1u);
            int32_t* gout = a.out_bucket ? a.out_bucket : a.out_phi;
            for (int l = 0; l < L; l++) {
                if (!(mask & (kmask << (l * k)))) continue;
                int gv = gout[row * L + l];
                for (int i = 0; i < k; i++) {
                    const int f = l * k + i;
                    if (mask & (1u << f)) {
                        const int b = 1 << (k - 1 - i);
                        gv = (bits >> f) & 1u ? (gv | b) : (gv & ~b);
                    }
                }
                if (a.out_phi) a.out_phi[row * L + l] = gv;
                if (a.out_bucket) a.out_bucket[row * L + l] = gv;
            }
        } else if (MODE == HM_CUBE_COSINE) {
            int vtx = a.out_h[row];
            for (int i = 0; i < k; i++)
                if (mask & (1u << i)) {
                    const int b = 1 << (k - 1 - i);
                    vtx = (bits >> i) & 1u ? (vtx | b) : (vtx & ~b);
                }
            a.out_h[row] = vtx;
        }
    }
}

int launch_hash_mfma(hipStream_t s, int mode, const float* X, int64_t N, const HashMfmaParams& p, int32_t* out_h,
                     int32_t* out_phi, int32_t* out_bucket, int32_t* mm, unsigned long long* list, int64_t list_cap,
                     int32_t* seg_counts, int seg_cap, unsigned long long* stats, int h16) {
    if (N <= 0) return 0;
    if (p.d != FU_D || p.LK > 32 || p.LK < 1 || !p.Vh || !p.Vl || !list || !seg_counts) {
        set_error("launch_hash_mfma: needs d = 128, 1 <= L*k <= 32 and the split image");
        return -1;
    }
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return kstatus("hipGetDevice");
    if (dev < 64 && !cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return kstatus("hipDeviceGetAttribute");
    const int ncu = dev < 64 && cus[dev] > 0 ? cus[dev] : 256;
    const int64_t ntiles = (N + 31) / 32;
    const int nblk = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)ncu * HMF_BPC, (ntiles + HMF_W - 1) / HMF_W));
    HashMfmaArgs a;
    a.X = X; a.N = N; a.Vh = p.Vh; a.Vl = p.Vl; a.tv = p.t; a.pnorm = p.pnorm; a.v1 = p.v1; a.rv = p.r; a.PT = p.PT;
    a.w = p.w; a.L = p.L; a.k = p.k; a.LK = p.LK; a.LKpad = p.LKpad; a.bdiv = make_bucket_div(p.nb);
    a.out_h = out_h; a.h16 = mode == HM_CUBE_EUCLID_H && h16; a.out_phi = out_phi; a.out_bucket = out_bucket; a.mm = mm;
    a.list = list; a.seg_counts = seg_counts; a.stats = stats;
    a.seg_rows = (int64_t)HMF_W * 32 * ((ntiles + (int64_t)nblk * HMF_W - 1) / ((int64_t)nblk * HMF_W));
    if (nblk > seg_cap || (int64_t)nblk * a.seg_rows > list_cap) {
        set_error("launch_hash_mfma: list workspace too small");
        return -1;
    }
    if ((mode == HM_LSH_EUCLID || mode == HM_CUBE_EUCLID_H) && !out_h) {
        set_error("launch_hash_mfma: the euclidean families need the h output");
        return -1;
    }
    if (mode == HM_CUBE_EUCLID_H && !mm) {
        set_error("launch_hash_mfma: the cube needs the h range output");
        return -1;
    }
    const dim3 grid((unsigned)nblk), block(64 * HMF_W);
    const dim3 fgrid((unsigned)nblk), fblock(HMF_FIX_THREADS);
    const size_t lds = hmf_lds_bytes();
    switch (mode) {
#define HMF_CASE(M)                                                                      \
    case M:                                                                              \
        hipLaunchKernelGGL(hash_mfma_kernel<M>, grid, block, lds, s, a);                 \
        hipLaunchKernelGGL(hash_mfma_fix_kernel<M>, fgrid, fblock, 0, s, a);             \
        break;
        HMF_CASE(HM_LSH_EUCLID) HMF_CASE(HM_LSH_COSINE) HMF_CASE(HM_CUBE_EUCLID_H) HMF_CASE(HM_CUBE_COSINE)
#undef HMF_CASE
        default:
            set_error("launch_hash_mfma: unknown mode");
            return -1;
    }
    return kstatus("hash_mfma.hip");
}

}  // namespace lshkm
