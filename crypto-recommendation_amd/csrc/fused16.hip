// fused16.hip — the hashing + Lloyd pass over 16-row tiles (v_mfma_f32_16x16x32_f16).
//
// The same one-read-of-X pass as fused_hi_kernel (fused.hip: EuclideanPhiGen::
// generate, euclidean_phi_gen.hpp:77-92, for L tables of k = 4 EuclideanH
// functions, euclidean_h_gen.hpp:73-76, and lloyds_assignment,
// assignment.hpp:54-80, with the certified f32 winner distance), laid out for
// occupancy: a wave holds 16 rows, lane (p, g) = (lane & 15, lane >> 4) the 32
// dims {32s + 8g .. 32s + 8g + 7 : s < 4} of row p -- half the row registers of
// the 32-row tile, so 16 waves (4 per SIMD) share one LDS image per CU.
//
// MFMA roles: D[c][p] = sum_k A[c][k] B[k][p] with A = 16 centroid rows from
// LDS (lane: row p of the tile, k-group g), B = the rows in registers, so lane
// (p, g) receives the scores of centroids 16t + 4g + r (r < 4) for its row p;
// the hash tile is the same with the 32 projection rows (two 16-row blocks:
// block b, k-group g = table 4b + g's four functions, k = 4).
//
// LDS image: centroid c's 16-B chunk q (dims 8q..8q+7) at c * 256 + 16 (q ^
// (c & 15)): the row reads of a ds_read_b128 lane group (lanes {0-3, 12-15,
// 20-27}, ...) hit 16 distinct 4-bank slots.
//
// Bounds: the centroid scores as fused_hi_kernel's (4 MFMAs of
// 32 products each, 128 additions into the -|c|^2/2 accumulator: FH_A); the
// hash tile's lo then hi products of a 32-dim step in one fresh accumulator (<=
// 32 roundings relative to the step's sum |terms|, the lo partials ~2^-11
// smaller), steps added in f32 (+3): 35.1 * 2^-23 = 1.10 * 2^-18, plus the
// split residual and lo terms (< 0.25 * 2^-18): F16_A1H = 1.375 * 2^-18.
// The winner distance: 4 fma per accumulator, a 3-level tree over 8, two
// cross-lane adds: <= 9 roundings (the 12 of the FAST bound hold).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "kernels.h"
#include "tile.h"
#include "fused_args.h"

namespace lshkm {

typedef float floatx4 __attribute__((ext_vector_type(4)));

#ifndef F16_WAVES_SET
#define F16_WAVES_SET 16
#endif
constexpr int F16_WAVES = F16_WAVES_SET;
#ifndef F16_TU
#define F16_TU 1        // centroid tiles per loop iteration (run-time tile count)
#endif
#ifndef F16_FIXNT
#define F16_FIXNT 1     // K = 256 / 512-centroid slices: the tile count compiled in
#endif
#ifndef F16_APF
#define F16_APF 0       // A-operand reads one tile ahead
#endif
#ifndef F16_FLOOR_SB
#define F16_FLOOR_SB 1
#endif
#ifndef F16_H64
#define F16_H64 0       // the f32 hash window's rejects refined in fp64 inside the pass
#endif
#ifndef F16_HASH_SB
#define F16_HASH_SB 1
#endif
constexpr int F16_RB = 256;                     // LDS bytes per image row (128 f16, swizzled chunks)
constexpr double F16_FH_A = 130.0 * 0x1p-23;
constexpr double F16_A1H = 1.375 * 0x1p-18;

__host__ __device__ constexpr int f16_lds_bytes(int Kpad, bool hash) {
    return 64 + Kpad * F16_RB + Kpad * 4 + (hash ? 2 * 32 * F16_RB + 4 * 32 * 4 : 0);
}
static_assert(f16_lds_bytes(512, true) <= 160 * 1024, "16-row form: LDS image exceeds 160 KiB");

// the other lane group's value: xor 16 (v_permlane16_swap) / xor 32
// (v_permlane32_swap); sums need no select (r[0] + r[1] = own + partner)
__device__ inline uint32_t x16_u(uint32_t v, int g) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (g & 1) ? r[0] : r[1];
}
__device__ inline uint32_t x32_u(uint32_t v, int g) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (g & 2) ? r[0] : r[1];
}
__device__ inline float sum4g(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float s = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ inline uint32_t or4g(uint32_t v) {
    const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    const uint32_t s = a[0] | a[1];
    const auto b = __builtin_amdgcn_permlane32_swap(s, s, false, false);
    return b[0] | b[1];
}
// fp64 sum over the row's 4 lane groups (the same value in all 4 lanes)
__device__ inline double sum4g_d(double v, int g) {
    const uint64_t u = __double_as_longlong(v);
    const double o1 = __longlong_as_double((long long)(((uint64_t)x16_u((uint32_t)(u >> 32), g) << 32) |
                                                       x16_u((uint32_t)u, g)));
    const double s = v + o1;
    const uint64_t w = __double_as_longlong(s);
    const double o2 = __longlong_as_double((long long)(((uint64_t)x32_u((uint32_t)(w >> 32), g) << 32) |
                                                       x32_u((uint32_t)w, g)));
    return s + o2;
}
__device__ inline float vmax3_16(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// MP (K > 512): one launch per 512-centroid slice a.Ch / a.cnh (slice offset
// 32 a.t0); hashing rides on the first, the certificate and the outputs on the
// last; between launches each row's merged (best, runner-up, index) crosses in
// a.part[row] (16 B).
// NTL: centroid tiles compiled in (16: K = 256, 32: a 512-centroid slice; the
// LDS offsets of the unrolled tile loop become immediates), 0: Kpad / 16 at run time
template <bool HASH, bool MP, int NTL>
__global__ __launch_bounds__(64 * F16_WAVES, 1) void fused16_kernel(FusedArgs a) {
    constexpr int NT = 64 * F16_WAVES;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int Kpad = a.Kpad;
    int* lcount = reinterpret_cast<int*>(smem);          // [0] uncertified rows, [1] hash fix-up rows
    char* lch = smem + 64;
    float* lcn = reinterpret_cast<float*>(lch + Kpad * F16_RB);
    char* lvh = reinterpret_cast<char*>(lcn + Kpad);
    char* lvl = lvh + 32 * F16_RB;
    float* lpn0 = reinterpret_cast<float*>(lvl + 32 * F16_RB);
    float* lv10 = lpn0 + 32;
    float* lt0 = lv10 + 32;
    int32_t* lr0 = reinterpret_cast<int32_t*>(lt0 + 32);
    const int tid = threadIdx.x;

    // centroid image (and the projections), 16-B granules, chunks swizzled
    {
        constexpr int CU = 4;
        const int ng = Kpad * 16;
        for (int e0 = 0; e0 < ng; e0 += NT * CU) {
            float4 v[CU];
#pragma unroll
            for (int u = 0; u < CU; u++) {
                const int e = e0 + u * NT + tid < ng ? e0 + u * NT + tid : 0;
                v[u] = *reinterpret_cast<const float4*>(a.Ch + (size_t)(e >> 4) * FU_D + (e & 15) * 8);
            }
#pragma unroll
            for (int u = 0; u < CU; u++) {
                const int e = e0 + u * NT + tid < ng ? e0 + u * NT + tid : 0;
                *reinterpret_cast<float4*>(lch + (e >> 4) * F16_RB + 16 * ((e & 15) ^ ((e >> 4) & 15))) = v[u];
            }
        }
        for (int e = tid; e < Kpad; e += NT) lcn[e] = a.cnh[e];
    }
    if (tid < 2) lcount[tid] = 0;
    if (HASH) {
        for (int e = tid; e < 32 * 16; e += NT) {
            const int r = e >> 4, q = e & 15;
            const int o = r * F16_RB + 16 * (q ^ (r & 15));
            *reinterpret_cast<float4*>(lvh + o) = *reinterpret_cast<const float4*>(a.Vh + r * FU_D + q * 8);
            *reinterpret_cast<float4*>(lvl + o) = *reinterpret_cast<const float4*>(a.Vl + r * FU_D + q * 8);
        }
        if (tid < 32) {
            const int f = tid;
            const bool on = f < a.LK;
            const double iwu = (double)(1.0f / a.w) * (1.0 + 0x1p-20);
            const double tf = on ? fabs((double)a.tv[f]) : 0.0;
            lpn0[f] = on ? (float)((F16_A1H * a.pnorm[f] * (1.0 + 0x1p-20) + FU_A2 * FU_SQRT_D) * iwu * (1.0 + 0x1p-18)) : 0.f;
            lv10[f] = on ? (float)((FU_A2 * a.v1[f] * (1.0 + 0x1p-20) + (0x1p-40 + 0x1p-23) * tf) * iwu * (1.0 + 0x1p-18) +
                                   0x1p-126) : 0.f;
            lt0[f] = on ? a.tv[f] : 0.f;
            lr0[f] = on ? a.rv[f] : 0;
        }
    }
    __syncthreads();

    const int lane = tid & 63, wave = tid >> 6;
    const int p = lane & 15, g = lane >> 4;
    const float cmaxf = a.cbound[3], crf = a.cbound[4], chf = a.cbound[5], cnf = a.cbound[6];
    const bool c_ok = __float_as_uint(a.cbound[2]) == 0u;
    const int ntl = NTL ? NTL : Kpad >> 4;
    const int64_t ntiles = (a.N + 15) >> 4;
    const double Ec = (0x1p-24 + F16_FH_A) * (double)cnf + 0x1p-41 * (double)cmaxf * (double)cmaxf + 0x1p-18 * (double)cnf;
    // this lane's A-operand offsets (row p of a 16-row block, chunk 4s + g)
    uint32_t ao[4];
#pragma unroll
    for (int s = 0; s < 4; s++) ao[s] = (uint32_t)(p * F16_RB + 16 * ((4 * s + g) ^ p));
    int32_t* ambig_seg = a.ambig + (int64_t)blockIdx.x * a.seg_rows;
    unsigned long long* hfix_seg = a.hfix + (int64_t)blockIdx.x * a.seg_rows;
    const int64_t tstride = (int64_t)gridDim.x * F16_WAVES;
    const bool first = !MP || a.pass_first != 0, last = !MP || a.pass_last != 0;
    const int c0 = MP ? 32 * a.t0 : 0;

    for (int64_t tile = (int64_t)blockIdx.x * F16_WAVES + wave; tile < ntiles; tile += tstride) {
        const int64_t row = tile * 16 + p;
        const bool valid = row < a.N;
        float xf[32];
        {
            const float* xr = a.X + (valid ? row : a.N - 1) * FU_D + 8 * g;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const float4 p0 = *reinterpret_cast<const float4*>(xr + 32 * s);
                const float4 p1 = *reinterpret_cast<const float4*>(xr + 32 * s + 4);
                xf[8 * s + 0] = p0.x; xf[8 * s + 1] = p0.y; xf[8 * s + 2] = p0.z; xf[8 * s + 3] = p0.w;
                xf[8 * s + 4] = p1.x; xf[8 * s + 5] = p1.y; xf[8 * s + 6] = p1.z; xf[8 * s + 7] = p1.w;
            }
        }
        half8 bh[4];
        float2v n2a = {0.f, 0.f}, n2b = {0.f, 0.f}, r2 = {0.f, 0.f};
        auto norms_step = [&](int s) {
#pragma unroll
            for (int j = 0; j < 8; j += 4) {
                const float2v u = {xf[8 * s + j], xf[8 * s + j + 1]}, v = {xf[8 * s + j + 2], xf[8 * s + j + 3]};
                n2a = __builtin_elementwise_fma(u, u, n2a);
                n2b = __builtin_elementwise_fma(v, v, n2b);
            }
        };
        floatx4 hs0, hs1;
        if (HASH) {
            // both 16-function blocks always (LK <= 16: block 1 unused; no branch in the step)
            constexpr bool two = true;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                half8 bl;
                split8_hi<true>(xf + 8 * s, bh[s], bl, r2);
                norms_step(s);
                const half8 ah = *reinterpret_cast<const half8*>(lvh + ao[s]);
                const half8 al = *reinterpret_cast<const half8*>(lvl + ao[s]);
                const floatx4 z = {};
                floatx4 t = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[s], z, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[s], t, 0, 0, 0);
                hs0 = s ? hs0 + t : t;
                if (two) {
                    const half8 ah1 = *reinterpret_cast<const half8*>(lvh + 16 * F16_RB + ao[s]);
                    const half8 al1 = *reinterpret_cast<const half8*>(lvl + 16 * F16_RB + ao[s]);
                    floatx4 t1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al1, bh[s], z, 0, 0, 0);
                    t1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah1, bl, t1, 0, 0, 0);
                    t1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah1, bh[s], t1, 0, 0, 0);
                    hs1 = s ? hs1 + t1 : t1;
                }
#if F16_HASH_SB
                __builtin_amdgcn_sched_barrier(0);    // keep the next step's LDS reads here (registers)
#endif
            }
        } else {
#pragma unroll
            for (int s = 0; s < 4; s++) {
                half8 unused;
                split8_hi<false>(xf + 8 * s, bh[s], unused, r2);
                norms_step(s);
            }
        }
        // |x|^2 and |x - xh|^2 over the row's 4 lane groups; f32 sums inflated
        // by 2^-16 (> d 2^-24): upper bounds
        const float xn2f = sum4g((n2a.x + n2a.y) + (n2b.x + n2b.y));
        const float xr2f = sum4g(r2.x + r2.y);
        const double xn2 = (double)xn2f * (1.0 + 0x1p-16);
        const double nx = sqrt(xn2);
        const double nxr = sqrt((double)xr2f * (1.0 + 0x1p-16)) + 0x1p-100;
        const double nxh = nx + nxr;
        const bool x_ok = xn2f <= FU_RANGE * FU_RANGE;

        if (HASH) {
            // floors of table 4b + g (functions 4(4b + g) + r in hs_b[r]), the
            // certificate of fused_hi_kernel with this tile's window
            uint32_t fmask = 0;
            if (!x_ok && valid) fmask = a.LK >= 32 ? 0xFFFFFFFFu : (1u << a.LK) - 1u;
            const float iw = 1.0f / a.w;
            const float nxf = (float)nx * (1.f + 0x1p-20f);
            constexpr float G = (0x1p-22f + 0x1p-20f) * (1.f + 0x1p-18f);
#pragma unroll
            for (int b = 0; b < 2; b++) {
                const int l = 4 * b + g;
                const bool on = l < a.L && valid;
                const int lc = on ? l : 0;
                const floatx4 hv4 = b ? hs1 : hs0;
                const float4 tq = *reinterpret_cast<const float4*>(lt0 + 4 * lc);
                const float4 pq = *reinterpret_cast<const float4*>(lpn0 + 4 * lc);
                const float4 qq = *reinterpret_cast<const float4*>(lv10 + 4 * lc);
                const int4 rq = *reinterpret_cast<const int4*>(lr0 + 4 * lc);
                const float tv[4] = {tq.x, tq.y, tq.z, tq.w}, pv[4] = {pq.x, pq.y, pq.z, pq.w};
                const float qv[4] = {qq.x, qq.y, qq.z, qq.w};
                const int32_t rv[4] = {rq.x, rq.y, rq.z, rq.w};
                int32_t hv[4];
                uint32_t fl = 0;                      // this table's uncertified functions
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float u = hv4[q] + tv[q];
                    const float y = u * iw;
                    const float B = fmaf(fabsf(y), G, fmaf(nxf, pv[q], qv[q]));
                    const float lo = floorf(y - B), hi = floorf(y + B);
                    hv[q] = (int32_t)lo;
                    if (lo != hi) fl |= 1u << q;
                }
                if (!on) fl = 0;
#if F16_H64
                // the f32 window's rejects redone in fp64 inside the pass (fix_row's
                // bound, hash_fixup_kernel): the row's 4 lanes form v_f . x over
                // their 32 dims (exact f32 products, 4 fp64 chains of 32 fma and
                // two adds), so only floors within ~2^-44 of an integer are listed
                uint32_t rm = x_ok ? or4g(fl << (4 * g)) : 0u;   // the same in the row's 4 lanes
                while (rm) {
                    const int fi = __builtin_ctz(rm);
                    rm &= rm - 1;
                    const int f = 16 * b + fi;
                    const float* vr = a.V32 + f * FU_D + 8 * g;
                    double acc = 0.0;
#pragma unroll
                    for (int s = 0; s < 4; s++) {
                        const float4 v0 = *reinterpret_cast<const float4*>(vr + 32 * s);
                        const float4 v1 = *reinterpret_cast<const float4*>(vr + 32 * s + 4);
                        const float vv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
                        for (int j = 0; j < 8; j++) acc = fma((double)vv[j], (double)xf[8 * s + j], acc);
                    }
                    acc = sum4g_d(acc, g);
                    const double P = a.pnorm[f] * nx * (1.0 + 0x1p-40);
                    const double tt = (double)a.tv[f], iwd = 1.0 / (double)a.w;
                    const double y = (acc + tt) * iwd;
                    const double B = ((double)(FU_D + 2) * 0x1p-52 * (P + fabs(tt))) * (iwd * (1.0 + 0x1p-50)) +
                                     fabs(y) * 0x1p-50;
                    const double lo = floor(y - B), hi = floor(y + B);
                    if (lo == hi && (fi >> 2) == g) {
#pragma unroll
                        for (int q = 0; q < 4; q++)
                            if (q == (fi & 3)) hv[q] = (int32_t)lo;
                        fl &= ~(1u << (fi & 3));
                    }
                }
#endif
                fmask |= fl << (4 * l);
                if (on) {
                    uint32_t hn = 0;
#pragma unroll
                    for (int q = 0; q < 4; q++) hn += phi_term_small(hv[q], rv[q]);
                    const int64_t o = row * a.L + l;
                    if (a.tuples) *reinterpret_cast<int4*>(a.tuples + o * 4) = make_int4(hv[0], hv[1], hv[2], hv[3]);
                    const uint32_t ph = phi_final(hn);
                    if (a.phi) a.phi[o] = (int32_t)ph;
                    if (a.bucket) a.bucket[o] = bucket_fast(ph, a.bdiv);
                }
#if F16_FLOOR_SB
                __builtin_amdgcn_sched_barrier(0);    // one table's constants live at a time
#endif
            }
            fmask = or4g(fmask);
            const unsigned long long fb = __ballot(fmask != 0u && g == 0);
            if (fb) {
                const int leader = __builtin_ctzll(fb);
                int base = 0;
                if (lane == leader) base = atomicAdd(lcount + 1, __popcll(fb));
                base = __shfl(base, leader);
                if (fmask != 0u && g == 0)
                    hfix_seg[base + __popcll(fb & ((1ull << lane) - 1ull))] = ((unsigned long long)row << 32) | fmask;
            }
        }

        // the certificate's bound E (the row's part; fused_hi_kernel's formula)
        const double E = (nxh * (double)crf + nxr * (double)cmaxf + F16_FH_A * nxh * (double)chf + 0x1p-41 * xn2 +
                          0x1p-18 * nx * (double)cmaxf + Ec) * (1.0 + 0x1p-20) + 1e-30;
        // ---- centroid tiles: 4 MFMAs each, accumulator initialised with -|c|^2/2;
        // each score carries r in its 2 low mantissa bits (the 2^-18 index term of E)
        float m1 = -__builtin_inff(), m2 = -__builtin_inff();
        int t1 = 0;
#if F16_APF
        // the next tile's A operand read as each step's register frees up
        half8 ab[4];
#pragma unroll
        for (int s = 0; s < 4; s++) ab[s] = *reinterpret_cast<const half8*>(lch + ao[s]);
#endif
        constexpr int UNR = NTL ? NTL : F16_TU;
#pragma unroll UNR
        for (int t = 0; t < (NTL ? NTL : ntl); t++) {
            const float m1p = m1;
            floatx4 acc = *reinterpret_cast<const floatx4*>(lcn + 16 * t + 4 * g);
#if F16_APF
            const char* an = lch + (t + 1 < ntl ? t + 1 : t) * 16 * F16_RB;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ab[s], bh[s], acc, 0, 0, 0);
                ab[s] = *reinterpret_cast<const half8*>(an + ao[s]);
            }
#else
            const char* at = lch + t * 16 * F16_RB;
#pragma unroll
            for (int s = 0; s < 4; s++)
                acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(*reinterpret_cast<const half8*>(at + ao[s]), bh[s], acc, 0, 0, 0);
#endif
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
                const float ta = __uint_as_float((__float_as_uint(acc[r]) & ~3u) | (uint32_t)r);
                const float tb = __uint_as_float((__float_as_uint(acc[r + 1]) & ~3u) | (uint32_t)(r + 1));
                m2 = __builtin_amdgcn_fmed3f(m2, __builtin_amdgcn_fmed3f(m1, ta, tb), 0x1.fffffep127f);
                m1 = vmax3_16(m1, ta, tb);
            }
            t1 = m1 != m1p ? t : t1;
        }
        // best and runner-up over the row's 4 lane groups (lowest index on ties)
        int i1 = c0 + t1 * 16 + 4 * g + (int)(__float_as_uint(m1) & 3u);
        {
            const float om1 = __uint_as_float(x16_u(__float_as_uint(m1), g));
            const float om2 = __uint_as_float(x16_u(__float_as_uint(m2), g));
            const int oi1 = (int)x16_u((uint32_t)i1, g);
            m2 = fmaxf(fmaxf(m2, om2), fminf(m1, om1));
            i1 = (om1 > m1 || (om1 == m1 && oi1 < i1)) ? oi1 : i1;
            m1 = fmaxf(m1, om1);
        }
        {
            const float om1 = __uint_as_float(x32_u(__float_as_uint(m1), g));
            const float om2 = __uint_as_float(x32_u(__float_as_uint(m2), g));
            const int oi1 = (int)x32_u((uint32_t)i1, g);
            m2 = fmaxf(fmaxf(m2, om2), fminf(m1, om1));
            i1 = (om1 > m1 || (om1 == m1 && oi1 < i1)) ? oi1 : i1;
            m1 = fmaxf(m1, om1);
        }
        if (MP && !first) {      // the earlier slices' state (lower indices: it wins ties)
            const float4 st = reinterpret_cast<const float4*>(a.part)[valid ? row : a.N - 1];
            const float om1 = st.x, om2 = st.y;
            const int oi1 = __float_as_int(st.z);
            m2 = fmaxf(fmaxf(m2, om2), fminf(m1, om1));
            i1 = (om1 > m1 || (om1 == m1 && oi1 < i1)) ? oi1 : i1;
            m1 = fmaxf(m1, om1);
        }
        if (MP && !last) {
            if (g == 0 && valid) reinterpret_cast<float4*>(a.part)[row] = make_float4(m1, m2, __int_as_float(i1), 0.f);
            continue;
        }
        const bool cert = x_ok && c_ok && ((double)m2 < (double)m1 - 2.0 * E);

        // certified f32 winner distance (fused_hi_kernel's FAST bound)
        const float* c32 = a.C32 + (size_t)i1 * FU_D + 8 * g;
        float2v q[4] = {};
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const float4 c0 = *reinterpret_cast<const float4*>(c32 + 32 * s);
            const float4 c1 = *reinterpret_cast<const float4*>(c32 + 32 * s + 4);
            const float2v cv[4] = {{c0.x, c0.y}, {c0.z, c0.w}, {c1.x, c1.y}, {c1.z, c1.w}};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float2v xv = {xf[8 * s + 2 * j], xf[8 * s + 2 * j + 1]};
                const float2v dv = xv - cv[j];
                q[j] = __builtin_elementwise_fma(dv, dv, q[j]);
            }
        }
        const float tq = sum4g(((q[0].x + q[0].y) + (q[1].x + q[1].y)) + ((q[2].x + q[2].y) + (q[3].x + q[3].y)));
        const double S = (double)tq, R = (double)a.rn32[i1];
        const double Bd = 14.2 * 0x1p-24 * S + 2.02 * R * sqrt(S) + 2.02 * R * R + 0x1p-100;
        const bool dok = Bd <= 0x1p-19 * S;                   // false for inf / nan
        const bool amb = valid && !(cert && dok);
        const unsigned long long amask = __ballot(amb && g == 0);
        if (amask) {
            const int leader = __builtin_ctzll(amask);
            int base = 0;
            if (lane == leader) base = atomicAdd(lcount, __popcll(amask));
            base = __shfl(base, leader);
            if (amb && g == 0) ambig_seg[base + __popcll(amask & ((1ull << lane) - 1ull))] = (int32_t)row;
        }
        if (g == 0 && valid && cert && dok) {
            a.assign[row] = i1;
            a.dist[row] = sqrt(S);
        }
    }
    __syncthreads();
    if (tid < 2 && (tid == 0 ? last : HASH)) {
        const int c = lcount[tid];
        a.seg_counts[2 * blockIdx.x + tid] = c;
        if (c) atomicAdd(tid == 0 ? a.ambig_count : a.hfix_count, (unsigned long long)c);
    }
}

int fused16_waves() { return F16_WAVES; }

// One launch over all rows for a slice of Kpad <= 512 centroids (euclidean,
// fp32 rows of 128 dims); mp: one of several slices (a.t0, a.pass_first,
// a.pass_last, a.part set by the caller; hash only with the first).
int launch_fused16(const FusedArgs& a, bool hash, bool mp, int nblk, hipStream_t s) {
    if (a.Kpad > 512 || (a.Kpad & 15) || !a.C32 || !a.rn32 || (hash && (a.k != 4 || a.LK > 32 || (F16_H64 && !a.V32))) ||
        (mp && (!a.part || (hash && !a.pass_first))))
        return -1;
    const size_t lds = (size_t)f16_lds_bytes(a.Kpad, hash);
    const dim3 grid((unsigned)nblk), block(64 * F16_WAVES);
#define F16_LAUNCH(H, M, T) hipLaunchKernelGGL((fused16_kernel<H, M, T>), grid, block, lds, s, a)
#define F16_BY_NT(H, M)                                      \
    do {                                                     \
        if (F16_FIXNT && a.Kpad == 256) F16_LAUNCH(H, M, 16); \
        else if (F16_FIXNT && a.Kpad == 512) F16_LAUNCH(H, M, 32); \
        else F16_LAUNCH(H, M, 0);                            \
    } while (0)
    if (mp) {
        if (hash) F16_BY_NT(true, true);
        else F16_BY_NT(false, true);
    } else {
        if (hash) F16_BY_NT(true, false);
        else F16_BY_NT(false, false);
    }
#undef F16_BY_NT
#undef F16_LAUNCH
    return 0;
}

}  // namespace lshkm
