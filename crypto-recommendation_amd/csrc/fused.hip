// fused.hip — one pass over the points: LSH hashing + Lloyd assignment on gfx950.
//
// Replaces, in one read of each point (SURVEY §8a rows a1-a3, a7's bucket ID,
// a12): EuclideanPhiGen::generate (lib/generators/euclidean_phi_gen.hpp:77-92)
// for L tables of k EuclideanH functions (euclidean_h_gen.hpp:73-76), and
// lloyds_assignment (lib/clustering_phases/assignment.hpp:54-80).
//
// Split-precision f16 MFMA. Every operand is split x = xh + xl (xh = f16(x),
// xl = f16(x - xh)); a dot product is sum(xh ch) [acc_hi] + sum(xh cl + xl ch)
// [acc_lo] on v_mfma_f32_32x32x16_f16: products of f16 values are exact in
// f32, and the separate hi accumulator keeps the rounding of the large terms
// at d ulps of f32. Rigorous bound on |dot~ - x.c|:
//   A1 |x||c| + A2 (|x|_1 + |c|_1),  A1 = 1.25 * 2^-16, A2 = 2^-24,
// which assumes nothing better than round-toward-zero accumulation. The f16
// range is guarded: a point with |x_j| > 2^15 (or non-finite) or a centroid set
// with |c_j| > 2^15 is never certified, so such inputs take the exact path.
//
// Block = 4 waves x 32 points. Wave w keeps its 32 points in registers as the
// B operand (lane half h holds dims 16s+8h..16s+8h+7 of point lane&31, hi and
// lo: 64 VGPRs); centroid hi/lo rows stream through LDS (64 per chunk, rows
// padded to 272 B: conflict-free ds_read_b128) as the A operand, so the tile
// D[centroid][point] has the point on the lane and the argmin is
// register-local. The hash projections are one extra 32-row tile.
// Per score: t = x.c - |c|^2/2 (argmax of t = argmin of the distance); the
// lane tracks the largest t (m1, index i1) and the runner-up m2. A point is
// certified iff m2 < m1 - 2E: then i1 is the reference's argmin, and its
// distance is recomputed in reference order (fp64 chain over j, sqrt).
// Otherwise the row goes to the exact all-centroid pass (assign.hip).
// Hash values: y = (dot~ + t)/w in fp64 with the split bound; a floor it
// cannot certify is redone from the exact row with the fp64 bound of
// hash.hip, and then, if needed, with the soft-x87 emulation.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <cstdio>

#include "common.h"
#include "kernels.h"
#include "softx87.h"
#include "exact.h"
#include "tile.h"
#include "fused_args.h"

namespace lshkm {

constexpr int FU_THREADS = 256;
constexpr int FU_PB = 128;               // points per block
constexpr int FU_CC = 64;                // centroids per LDS chunk
constexpr int FU_CH_BYTES = FU_CC * FU_RS * 2;          // one of hi / lo
constexpr int FU_CHUNK_BYTES = 2 * FU_CH_BYTES + FU_CC * 4;
constexpr int FU_XSTAGE_BYTES = 4 * 32 * FU_D * 4;      // 64 KiB (aliases the chunk region)
constexpr int FU_HS_OFF = FU_XSTAGE_BYTES;              // hash values [128][32] int32
constexpr int FU_LDS_BYTES = FU_HS_OFF + FU_PB * 32 * 4; // 80 KiB -> 2 blocks / CU
static_assert(FU_CHUNK_BYTES <= FU_XSTAGE_BYTES, "chunk region must fit in the staging alias");


// Profiling builds (make prof -> liblshkm_prof.so) accumulate s_memtime per
// phase of the persistent loop; the product library compiles these away.
#ifdef LSHKM_PHASE_TIMING
#define PT_DECL unsigned long long pt_acc[6] = {0, 0, 0, 0, 0, 0}; unsigned long long pt_t = __builtin_amdgcn_s_memtime();
#define PT_MARK(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); pt_acc[i] += t_ - pt_t; pt_t = t_; }
#define PT_FLUSH if (lane == 0) for (int i_ = 0; i_ < 6; i_++) atomicAdd(a.prof + i_, pt_acc[i_]);
#elif defined(LSHKM_ISA_MARK)       // assembly listings: region comments (tools/isa_regions.py)
#define PT_DECL
#define PT_MARK(i) asm volatile(";PTMARK " #i);
#define PT_FLUSH
#else
#define PT_DECL
#define PT_MARK(i)
#define PT_FLUSH
#endif

__device__ inline void split8(const float* x, half8& hi, half8& lo) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const _Float16 hv = (_Float16)x[j];
        hi[j] = hv;
        lo[j] = (_Float16)(x[j] - (float)hv);
    }
}

// split8 in 2 VALU per element: v_cvt_pk_f16_f32 (hi pair), two residuals by
// v_fma_mix_f32, v_cvt_pk_f16_f32 (lo pair).
__device__ inline void split8p(const float* x, half8& hi, half8& lo) {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        const half2v hp = {(_Float16)x[j], (_Float16)x[j + 1]};
        hi[j] = hp.x;
        hi[j + 1] = hp.y;
        const half2v lp = {(_Float16)resid_lo(x[j], hp), (_Float16)resid_hi(x[j + 1], hp)};
        lo[j] = lp.x;
        lo[j + 1] = lp.y;
    }
}

// Within each group of 4 lanes, lane q receives lane q-1's value (lane 0 its
// own): DPP quad_perm [0,0,1,2], a VALU move.
__device__ inline double quad_shift_up(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, 0x90, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), 0x90, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

// __shfl_xor(v, 32) as two v_permlane32_swap (gfx950 VALU lane-half swap)
// instead of two LDS bpermutes: sw[0] holds the lower half's value in the
// upper lanes, sw[1] the upper half's value in the lower lanes.
__device__ inline double swap_halves(double v, int h) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
    const uint32_t l = h ? lo[0] : lo[1], u = h ? hi[0] : hi[1];
    return __longlong_as_double((long long)(((uint64_t)u << 32) | l));
}

__device__ inline float swap_halves_f(float v, int h) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(h ? r[0] : r[1]);
}

// One direction of the half swap (the chain hand-offs): take_from_lower gives
// the upper lanes the lower half's value and leaves the lower lanes' own (the
// first result of v_permlane32_swap(v, v)); take_from_upper the other way.
// No select: one v_permlane32_swap per dword.
__device__ inline double take_from_lower(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t l = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false)[0];
    const uint32_t u = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false)[0];
    return __longlong_as_double((long long)(((uint64_t)u << 32) | l));
}
__device__ inline double take_from_upper(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t l = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false)[1];
    const uint32_t u = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false)[1];
    return __longlong_as_double((long long)(((uint64_t)u << 32) | l));
}

// Exact (reference-order) hash of one projection from the fp32 row in HBM.
__device__ int32_t hash_exact_row(const float* __restrict__ xrow, const double* __restrict__ PT, int LKpad, int f,
                                  float t, float w, double pn, unsigned long long* stats) {
    double acc = 0.0, xn2 = 0.0;
    for (int j = 0; j < FU_D; j++) {
        const double xj = (double)xrow[j];
        xn2 = fma(xj, xj, xn2);
        acc = fma(PT[(size_t)j * LKpad + f], xj, acc);
    }
    const double P = pn * sqrt(xn2) * (1.0 + 0x1p-40);
    const double tt = (double)t, ww = (double)w;
    const double y = (acc + tt) / ww;
    const double B = ((double)(FU_D + 2) * 0x1p-52 * (P + fabs(tt))) / ww + fabs(y) * 0x1p-51;
    const double lo = floor(y - B), hi = floor(y + B);
    if (lo == hi) return (int32_t)lo;
    sx80 s = sx_zero();
    for (int j = 0; j < FU_D; j++) s = sx_add_double(s, __dmul_rn(PT[(size_t)j * LKpad + f], (double)xrow[j]));
    s = sx_add_double(s, tt);
    atomicAdd(stats + STAT_HASH_EXACT, 1ull);
    return (int32_t)sx_floor_i64(sx_div(s, sx_from_float(w)));
}

// Load rows [r0, r0 + 64) of a [rows][128] f16 matrix into the padded LDS image.
__device__ inline void load_rows_f16(const _Float16* __restrict__ src, int r0, _Float16* dst) {
    // 64 rows x 16 granules of 16 B, 256 threads -> 4 granules each
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int e = threadIdx.x + u * FU_THREADS;
        const int row = e >> 4, g = e & 15;
        const float4 v = *reinterpret_cast<const float4*>(src + (size_t)(r0 + row) * FU_D + g * 8);
        *reinterpret_cast<float4*>(dst + row * FU_RS + g * 8) = v;
    }
}

// One 32-row tile: acc_hi = sum(Ah Bh), acc_lo = sum(Ah Bl + Al Bh).
__device__ inline void tile_mfma(const _Float16* ah_row, const _Float16* al_row, const half8 (&bh)[8],
                                 const half8 (&bl)[8], floatx16& acc_hi, floatx16& acc_lo) {
#pragma unroll
    for (int r = 0; r < 16; r++) { acc_hi[r] = 0.f; acc_lo[r] = 0.f; }
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const half8 ah = *reinterpret_cast<const half8*>(ah_row + 16 * s);
        const half8 al = *reinterpret_cast<const half8*>(al_row + 16 * s);
        acc_hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc_hi, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], acc_lo, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s], acc_lo, 0, 0, 0);
    }
}

template <bool HASH>
__global__ __launch_bounds__(FU_THREADS, 2) void fused_kernel(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 31, h = lane >> 5;
    const int lp = wave * 32 + col;                         // point within the block
    const int64_t pbase = (int64_t)blockIdx.x * FU_PB + wave * 32;
    const int64_t row = pbase + col;
    const bool valid = row < a.N;

    // ---- phase 0: stage this wave's 32 rows (XOR-swizzled 16-B granules), split to f16
    float* xs = reinterpret_cast<float*>(smem) + wave * 32 * FU_D;
    for (int e = lane; e < 32 * (FU_D / 4); e += 64) {
        const int r = e >> 5, g = e & 31;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (pbase + r < a.N) v = *reinterpret_cast<const float4*>(a.X + (pbase + r) * FU_D + g * 4);
        *reinterpret_cast<float4*>(xs + r * FU_D + 4 * (g ^ (r & 15))) = v;
    }
    __syncthreads();
    half8 bh[8], bl[8];
    float xn2f = 0.f, x1f = 0.f, xmax = 0.f;
#pragma unroll
    for (int s = 0; s < 8; s++) {
        float xv[8];
        const int g0 = 4 * s + 2 * h;                       // granules of dims 16s+8h .. +7
        const float4 p0 = *reinterpret_cast<const float4*>(xs + col * FU_D + 4 * (g0 ^ (col & 15)));
        const float4 p1 = *reinterpret_cast<const float4*>(xs + col * FU_D + 4 * ((g0 + 1) ^ (col & 15)));
        xv[0] = p0.x; xv[1] = p0.y; xv[2] = p0.z; xv[3] = p0.w;
        xv[4] = p1.x; xv[5] = p1.y; xv[6] = p1.z; xv[7] = p1.w;
        split8(xv, bh[s], bl[s]);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            xn2f = fmaf(xv[j], xv[j], xn2f);
            x1f += fabsf(xv[j]);
            xmax = fmaxf(xmax, fabsf(xv[j]));
        }
    }
    xn2f += __shfl_xor(xn2f, 32);
    x1f += __shfl_xor(x1f, 32);
    xmax = fmaxf(xmax, __shfl_xor(xmax, 32));
    // f32 sums of squares/abs: inflate by (1 + 2^-16) (> d * 2^-24) to stay upper bounds
    const double xn2 = (double)xn2f * (1.0 + 0x1p-16);
    const double nx = sqrt(xn2);
    const double x1 = (double)x1f * (1.0 + 0x1p-16);
    const bool x_ok = xmax <= FU_RANGE;                    // false for inf / nan too
    __syncthreads();                                       // staging area becomes the chunk region

    _Float16* lch = reinterpret_cast<_Float16*>(smem);
    _Float16* lcl = reinterpret_cast<_Float16*>(smem + FU_CH_BYTES);
    float* lcn = reinterpret_cast<float*>(smem + 2 * FU_CH_BYTES);
    int32_t* hs = reinterpret_cast<int32_t*>(smem + FU_HS_OFF);
    const _Float16* my_h = lch + col * FU_RS + 8 * h;      // A rows of this lane (tile 0)
    const _Float16* my_l = lcl + col * FU_RS + 8 * h;

    // ---- hash tile (projections as 32 extra rows)
    if (HASH) {
        load_rows_f16(a.Vh, 0, lch);
        load_rows_f16(a.Vl, 0, lcl);   // rows 32..63 of the image are unused here
        __syncthreads();
        floatx16 acc_hi, acc_lo;
        tile_mfma(my_h, my_l, bh, bl, acc_hi, acc_lo);
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int f = (r & 3) + 8 * (r >> 2) + 4 * h;
            if (f >= a.LK || !valid) continue;
            const float dotf = acc_hi[r] + acc_lo[r];
            const double tt = (double)a.tv[f], ww = (double)a.w;
            const double y = ((double)dotf + tt) / ww;
            const double Ed = FU_A1 * a.pnorm[f] * nx + FU_A2 * (a.v1[f] + x1) + 0x1p-23 * fabs((double)dotf);
            const double B = (Ed + 0x1p-50 * (a.pnorm[f] * nx + fabs(tt))) / ww + fabs(y) * 0x1p-50;
            const double lo = floor(y - B), hi = floor(y + B);
            int32_t hv;
            if (lo == hi && x_ok) hv = (int32_t)lo;
            else hv = hash_exact_row(a.X + row * FU_D, a.PT, a.LKpad, f, a.tv[f], a.w, a.pnorm[f], a.stats);
            hs[lp * 32 + f] = hv;
        }
        __syncthreads();
    }

    // ---- centroid chunks
    const float ecf = a.cbound[0], ebf = a.cbound[1];
    const bool c_ok = __float_as_uint(a.cbound[2]) == 0u;
    const float E = (float)(nx * (double)ecf + (double)ebf + FU_A2 * x1 + 0x1p-41 * xn2) * (1.f + 0x1p-20f) + 1e-30f;
    float m1 = -__builtin_inff(), m2 = -__builtin_inff();
    int i1 = 0;
    for (int c0 = 0; c0 < a.Kpad; c0 += FU_CC) {
        load_rows_f16(a.Ch, c0, lch);
        load_rows_f16(a.Cl, c0, lcl);
        if (threadIdx.x < FU_CC) lcn[threadIdx.x] = a.cnh[c0 + threadIdx.x];
        __syncthreads();
#pragma unroll 1
        for (int t = 0; t < FU_CC / 32; t++) {
            floatx16 acc_hi, acc_lo;
            tile_mfma(my_h + t * 32 * FU_RS, my_l + t * 32 * FU_RS, bh, bl, acc_hi, acc_lo);
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int cb = t * 32 + 8 * g + 4 * h;     // D rows of registers 4g..4g+3
                const float4 cn = *reinterpret_cast<const float4*>(lcn + cb);
                const float cnv[4] = {cn.x, cn.y, cn.z, cn.w};
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float tv = (acc_hi[4 * g + q] + acc_lo[4 * g + q]) + cnv[q];
                    m2 = fmaxf(m2, fminf(m1, tv));
                    const bool c1 = tv > m1;
                    m1 = c1 ? tv : m1;
                    i1 = c1 ? c0 + cb + q : i1;
                }
            }
        }
        __syncthreads();
    }

    // ---- merge the two lane halves of each point, certify
    const float om1 = __shfl_xor(m1, 32), om2 = __shfl_xor(m2, 32);
    const int oi1 = __shfl_xor(i1, 32);
    const float M2 = fmaxf(fmaxf(m2, om2), fminf(m1, om1));
    const int I1 = (om1 > m1 || (om1 == m1 && oi1 < i1)) ? oi1 : i1;
    const float M1 = fmaxf(m1, om1);
    const bool cert = x_ok && c_ok && ((double)M2 < (double)M1 - 2.0 * (double)E);

    // ---- exact-order distance of the winner: lane h=0 dims [0,64), lane h=1 [64,128)
    double accd = 0.0;
    const float* xrow = a.X + row * FU_D;
    if (h == 0 && cert && valid) {
        const double* crow = a.C64 + (size_t)I1 * FU_D;
        for (int j = 0; j < FU_D / 2; j++) {
            const double df = __dsub_rn((double)xrow[j], crow[j]);
            accd = __dadd_rn(accd, gp_sq(df));
        }
    }
    const double part = __shfl_xor(accd, 32);
    if (h == 1 && valid) {
        if (cert) {
            double s2 = part;
            const double* crow = a.C64 + (size_t)I1 * FU_D;
            for (int j = FU_D / 2; j < FU_D; j++) {
                const double df = __dsub_rn((double)xrow[j], crow[j]);
                s2 = __dadd_rn(s2, gp_sq(df));
            }
            a.assign[row] = I1;
            a.dist[row] = sqrt(s2);
        } else {
            const unsigned long long slot = atomicAdd(a.ambig_count, 1ull);
            a.ambig[slot] = (int32_t)row;
        }
    }

    // ---- LSH outputs: tuples, phi, bucket ids (euclidean_phi_gen.hpp:77-92, cust_hashtable.hpp:68)
    if (HASH) {
        const int64_t p0 = (int64_t)blockIdx.x * FU_PB;
        const int npts = (int)min((int64_t)FU_PB, a.N - p0);
        const int LK = a.LK, L = a.L, k = a.k;
        if (a.tuples)
            for (int e = threadIdx.x; e < npts * LK; e += FU_THREADS) {
                const int pp = e / LK, f = e - pp * LK;
                a.tuples[p0 * LK + e] = hs[pp * 32 + f];
            }
        const int64_t M = 2147483647;   // int(pow(2,32)-5) under g++ (euclidean_phi_gen.hpp:70)
        for (int q = threadIdx.x; q < npts * L; q += FU_THREADS) {
            const int pp = q / L, l = q - pp * L;
            uint32_t hn = 0;
            for (int i = 0; i < k; i++) {
                const int hi = hs[pp * 32 + l * k + i];
                const int64_t temp = (int64_t)(int32_t)((uint32_t)hi * (uint32_t)a.rv[l * k + i]);
                hn += (uint32_t)(int32_t)((temp % M + M) % M);
            }
            const uint32_t ph = (hn % 2147483647u + 2147483647u) % 2147483647u;
            if (a.phi) a.phi[p0 * L + q] = (int32_t)ph;
            if (a.bucket) a.bucket[p0 * L + q] = (int32_t)((uint64_t)ph % (uint64_t)a.nb);
        }
    }
}

// ------------------------------------------------------------- persistent form
// For Kpad <= 256 the whole split centroid set (2 x 256 x 272 B) fits in LDS
// next to the 32 hash rows, so one block per CU loads it ONCE and its 8 waves
// (2 per SIMD) then loop independently over 32-point tiles: no barrier in the
// main loop, points go straight from HBM into registers (lane half h: dims
// 16s+8h..+7 of point lane&31 -- the B-operand layout) and stay there, exact,
// for the winner's reference-order distance. Hashing here is
// specialised to k = 4 (the reference default, euclidean_phi_gen.hpp): table l's
// four values are then D-registers 4(l>>1)..+3 of lane half l&1, so phi and the
// bucket ID are computed in-register.
// FP_KEEP_X (default): the exact row stays in registers for the distance chain,
// 8 waves/CU. 0: 12 waves/CU re-reading the row in a quad layout -- measured
// 18% slower, the re-read mostly misses L2 (12 x 16 KiB in flight per CU).
#ifndef FP_KEEP_X
#define FP_KEEP_X 1
#endif
// FP_WAVES_SET = 4 (one wave per SIMD, 512 registers, TILE_UNROLL 8): measured
// 3.50 ms vs 2.93 -- the second wave's overlap is worth more than the registers.
#ifndef FP_WAVES_SET
#define FP_WAVES_SET 0
#endif
constexpr int FP_WAVES = FP_WAVES_SET ? FP_WAVES_SET : FP_KEEP_X ? 8 : 12;   // 2 / 3 per SIMD: <= 256 / 168 VGPRs
#ifndef TILE_UNROLL
#define TILE_UNROLL 1
#endif
#ifndef MFMA_PRIO
#define MFMA_PRIO 1     // s_setprio inside the centroid loop (measured +1-3%)
#endif
#ifndef CHAIN_PRIO
#define CHAIN_PRIO 2    // s_setprio around the hi-only kernel's winner chain (measured -0.02 ms; 0 = off)
#endif
#ifndef YOUNG_PRIO
#define YOUNG_PRIO 0    // s_setprio for waves FP_WAVES/2.. for the whole loop (experiment knob)
#endif
#ifndef PIPE_TILES
#define PIPE_TILES 0    // 1: measured 3.13 ms vs 2.91 (WAVE_OFFSET 8: 2.96, TILE_UNROLL 2: 2.91)
#endif
// Winner-row loads of the distance chain issued CHAIN_PF 16-dim steps ahead.
// Measured (fused pass, N = 10M): 1 -> 3.03 ms, 2 -> 3.11, 4 -> 3.16, 8 -> 3.32:
// the chain's L2 round trips are not what limits the pass (the SIMDs' VALU +
// MFMA issue is), and the prefetch registers cost more than they hide.
#ifndef CHAIN_PF
#define CHAIN_PF 1
#endif
#ifndef XPF
#define XPF 0           // hi-only kernel: next tile's row loaded during the winner chain
#endif
// General rows (ROWS = 1: fp32, 2: fp64; d <= 128 dims, row stride d): lane
// half h's 64 values of row rowc in the B-operand layout (dims 16s+8h..+7),
// zero past d; fp64 values rounded to f32 (the scores' operand; the bounds add
// |x - f32(x)| <= 2^-24 |x|).
template <int ROWS>
__device__ inline void load_row_gen(const FusedArgs& a, int64_t rowc, int h, float (&dst)[64]) {
    const int64_t ro = rowc * (int64_t)a.d;
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const int j0 = 16 * s + 8 * h;
        if (a.xvec && j0 + 8 <= a.d) {
            if constexpr (ROWS == 1) {
                const float4 p0 = *reinterpret_cast<const float4*>(a.X + ro + j0);
                const float4 p1 = *reinterpret_cast<const float4*>(a.X + ro + j0 + 4);
                dst[8 * s + 0] = p0.x; dst[8 * s + 1] = p0.y; dst[8 * s + 2] = p0.z; dst[8 * s + 3] = p0.w;
                dst[8 * s + 4] = p1.x; dst[8 * s + 5] = p1.y; dst[8 * s + 6] = p1.z; dst[8 * s + 7] = p1.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const double2 q = *reinterpret_cast<const double2*>(a.X64 + ro + j0 + 2 * j);
                    dst[8 * s + 2 * j] = (float)q.x;
                    dst[8 * s + 2 * j + 1] = (float)q.y;
                }
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; e++) {
                float v = 0.f;
                if (j0 + e < a.d) v = ROWS == 1 ? a.X[ro + j0 + e] : (float)a.X64[ro + j0 + e];
                dst[8 * s + e] = v;
            }
        }
    }
}
// fp64 rows: the exact values of 16-dim step st of lane half h (the winner chain)
__device__ inline void load_x64_step(const FusedArgs& a, int64_t rowc, int st, int h, double2 (&o)[4]) {
    const int64_t ro = rowc * (int64_t)a.d;
    const int j0 = 16 * st + 8 * h;
    if (a.xvec && j0 + 8 <= a.d) {
#pragma unroll
        for (int j = 0; j < 4; j++) o[j] = *reinterpret_cast<const double2*>(a.X64 + ro + j0 + 2 * j);
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            o[j] = make_double2(0.0, 0.0);
            if (j0 + 2 * j < a.d) o[j].x = a.X64[ro + j0 + 2 * j];
            if (j0 + 2 * j + 1 < a.d) o[j].y = a.X64[ro + j0 + 2 * j + 1];
        }
    }
}

// hi-only kernel's winner-row loads
#define CHAIN_LD(ptr, xi) (*reinterpret_cast<const double2*>(ptr))

// Scores of one 32-centroid tile: t = (hi + lo) + (-|c|^2/2) on packed f32
// (D rows of registers 4g..4g+3 are centroids 8g+4h..+3 of the tile).
__device__ inline void tile_scores(const floatx16& acc_hi, const floatx16& acc_lo, const float* cn_tile_h,
                                   float (&sv)[16]) {
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const float4 cn = *reinterpret_cast<const float4*>(cn_tile_h + 8 * g);
        const float2v h01 = {acc_hi[4 * g], acc_hi[4 * g + 1]}, l01 = {acc_lo[4 * g], acc_lo[4 * g + 1]};
        const float2v h23 = {acc_hi[4 * g + 2], acc_hi[4 * g + 3]}, l23 = {acc_lo[4 * g + 2], acc_lo[4 * g + 3]};
        const float2v c01 = {cn.x, cn.y}, c23 = {cn.z, cn.w};
        const float2v s01 = (h01 + l01) + c01, s23 = (h23 + l23) + c23;
        sv[4 * g] = s01.x; sv[4 * g + 1] = s01.y; sv[4 * g + 2] = s23.x; sv[4 * g + 3] = s23.y;
    }
}

// One accumulator per tile (ONE_ACC): the lo products first (their partial sums
// stay below 2^-10 |x||c|, so their <= 256 roundings add < 2^-25 |x||c|), then
// the 8 hi MFMAs continue the same chain (<= 128 roundings of sum |terms|, as
// acc_hi had): A1 still bounds the error, and the hi + lo add disappears.
__device__ inline void tile_mfma1(const _Float16* ah_row, const _Float16* al_row, const half8 (&bh)[8],
                                  const half8 (&bl)[8], floatx16& acc) {
    const floatx16 z = {};
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const half8 ah = *reinterpret_cast<const half8*>(ah_row + 16 * s);
        const half8 al = *reinterpret_cast<const half8*>(al_row + 16 * s);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], s ? acc : z, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s], acc, 0, 0, 0);
    }
#pragma unroll
    for (int s = 0; s < 8; s++) {
        const half8 ah = *reinterpret_cast<const half8*>(ah_row + 16 * s);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc, 0, 0, 0);
    }
}
__device__ inline void tile_scores1(const floatx16& acc, const float* cn_tile_h, float (&sv)[16]) {
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const float4 cn = *reinterpret_cast<const float4*>(cn_tile_h + 8 * g);
        const float2v a01 = {acc[4 * g], acc[4 * g + 1]}, a23 = {acc[4 * g + 2], acc[4 * g + 3]};
        const float2v c01 = {cn.x, cn.y}, c23 = {cn.z, cn.w};
        const float2v s01 = a01 + c01, s23 = a23 + c23;
        sv[4 * g] = s01.x; sv[4 * g + 1] = s01.y; sv[4 * g + 2] = s23.x; sv[4 * g + 3] = s23.y;
    }
}
#ifndef ONE_ACC
#define ONE_ACC 0       // measured: 2.95 ms vs 2.91 with two accumulators (A/B on one box)
#endif

// Running best / runner-up over one tile's scores. Each score carries its
// in-tile index (4g+q) in its low 4 mantissa bits (see E), so the best needs
// no compare/select per score. Per pair (ta, tb) of new scores:
//   m2 = max(m2, med3(m1, ta, tb)),  m1 = max3(m1, ta, tb)
// (the runner-up of {m1 >= m2, ta, tb} is the larger of m2 and the median of
// the other three): 3 VALU per 2 scores. v_max3 / v_med3 as instructions:
// fmaxf would first re-quiet its operands (IEEE mode); scores are finite for
// any certifiable point.
__device__ inline float vmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
#ifndef EPI_MAX3
#define EPI_MAX3 1
#endif
__device__ inline void tile_epilogue(const float (&sv)[16], float& m1, float& m2) {
#if EPI_MAX3
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
        const float ta = __uint_as_float((__float_as_uint(sv[r]) & ~0xFu) | (uint32_t)r);
        const float tb = __uint_as_float((__float_as_uint(sv[r + 1]) & ~0xFu) | (uint32_t)(r + 1));
        m2 = __builtin_amdgcn_fmed3f(m2, __builtin_amdgcn_fmed3f(m1, ta, tb), 0x1.fffffep127f);
        m1 = vmax3(m1, ta, tb);
    }
#else
    // two independent (best, runner-up) chains over the even / odd scores,
    // merged at the end; max(a, b) as med3(a, b, FLT_MAX)
    float a1 = m1, a2 = m2, b1 = -__builtin_inff(), b2 = -__builtin_inff();
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
        const float ta = __uint_as_float((__float_as_uint(sv[r]) & ~0xFu) | (uint32_t)r);
        const float tb = __uint_as_float((__float_as_uint(sv[r + 1]) & ~0xFu) | (uint32_t)(r + 1));
        a2 = __builtin_amdgcn_fmed3f(a2, a1, ta);
        a1 = __builtin_amdgcn_fmed3f(a1, ta, 0x1.fffffep127f);
        b2 = __builtin_amdgcn_fmed3f(b2, b1, tb);
        b1 = __builtin_amdgcn_fmed3f(b1, tb, 0x1.fffffep127f);
    }
    m2 = __builtin_amdgcn_fmed3f(__builtin_amdgcn_fmed3f(a2, b2, 0x1.fffffep127f), __builtin_amdgcn_fmed3f(a1, b1, -0x1.fffffep127f), 0x1.fffffep127f);
    m1 = __builtin_amdgcn_fmed3f(a1, b1, 0x1.fffffep127f);
#endif
}
constexpr int FP_THREADS = 64 * FP_WAVES;
constexpr int FP_KMAX = 256;
constexpr int FP_HC_BYTES = 32 * (4 + 4 + 4 + 4);     // hash constants |v|_2, |v|_1, t, r

__host__ __device__ constexpr int fp_lds_bytes(int Kpad, bool hash) {
    return 16 + 2 * Kpad * FU_RS * 2 + Kpad * 4 + (hash ? 2 * 32 * FU_RS * 2 + FP_HC_BYTES : 0);
}
static_assert(fp_lds_bytes(FP_KMAX, true) <= 160 * 1024, "persistent LDS image exceeds 160 KiB");

// MET = 1: cosine Lloyd (HASH = false): centroids are normalised in the prep
// (score x.c/|c|, cnh = 0), the winner distance is exact.h's certified form.
// MP: multi-pass (K > 256) form; the single-pass instantiation compiles without
// the pass-state code. LIST: the rows are block b's segment of a row list (the
// refinement of fused_hi_kernel's uncertified rows), not a range.
// ROWS = 1 / 2 (LIST only): the refinement of fused_hi_kernel<..., ROWS>'s rows
// (general rows, see there); fp64 rows add |x - f32(x)| |c| <= 2^-24 |x| |c| to E.
template <bool HASH, int MET = 0, bool MP = false, bool LIST = false, int ROWS = 0>
__global__ __launch_bounds__(FP_THREADS, 1) void fused_persistent_kernel(FusedArgs a) {
    static_assert(ROWS == 0 || (LIST && !HASH && FP_KEEP_X), "general rows: the LIST form");
    static_assert(FP_KEEP_X || !LIST, "the quad-layout chain re-reads rows by tile index");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int Kpad = a.Kpad;
    int* lcount = reinterpret_cast<int*>(smem);          // [0] ambiguous rows, [1] hash fix-up rows
    _Float16* lch = reinterpret_cast<_Float16*>(smem + 16);
    _Float16* lcl = lch + Kpad * FU_RS;
    float* lcn = reinterpret_cast<float*>(lcl + Kpad * FU_RS);
    _Float16* lvh = reinterpret_cast<_Float16*>(lcn + Kpad);
    _Float16* lvl = lvh + 32 * FU_RS;
    float* lpn0 = reinterpret_cast<float*>(lvl + 32 * FU_RS);
    float* lv10 = lpn0 + 32;
    float* lt0 = lv10 + 32;
    int32_t* lr0 = reinterpret_cast<int32_t*>(lt0 + 32);

    // ---- prologue: the block's resident image (once per block), FP_CU granules
    // per thread in flight at once (a plain copy loop waited on every load)
    constexpr int FP_CU = 4;
    for (int e0 = 0; e0 < Kpad * 16; e0 += FP_THREADS * FP_CU) {
        float4 vh[FP_CU], vl[FP_CU];
#pragma unroll
        for (int u = 0; u < FP_CU; u++) {
            // past the end: granule 0 again (the same bytes rewritten), so neither
            // the loads nor the stores carry a branch and the loads issue together
            const int e = e0 + u * FP_THREADS + (int)threadIdx.x < Kpad * 16 ? e0 + u * FP_THREADS + (int)threadIdx.x : 0;
            const int r = e >> 4, g = e & 15;
            vh[u] = *reinterpret_cast<const float4*>(a.Ch + (size_t)r * FU_D + g * 8);
            vl[u] = *reinterpret_cast<const float4*>(a.Cl + (size_t)r * FU_D + g * 8);
        }
#pragma unroll
        for (int u = 0; u < FP_CU; u++) {
            const int e = e0 + u * FP_THREADS + (int)threadIdx.x < Kpad * 16 ? e0 + u * FP_THREADS + (int)threadIdx.x : 0;
            const int r = e >> 4, g = e & 15;
            *reinterpret_cast<float4*>(lch + r * FU_RS + g * 8) = vh[u];
            *reinterpret_cast<float4*>(lcl + r * FU_RS + g * 8) = vl[u];
        }
    }
    for (int e = threadIdx.x; e < Kpad; e += FP_THREADS) lcn[e] = a.cnh[e];
    if (threadIdx.x < 2) lcount[threadIdx.x] = 0;
    // This block's list segments (no device-wide atomic in the loop: a contended
    // global counter serialises at ~12 ns per add, MI355X_MICROARCH.md "fanin").
    int32_t* ambig_seg = a.ambig + (int64_t)blockIdx.x * a.seg_rows;
    unsigned long long* hfix_seg = a.hfix + (int64_t)blockIdx.x * a.seg_rows;
    if (HASH) {
        for (int e = threadIdx.x; e < 32 * 16; e += FP_THREADS) {   // 32 rows x 16 granules
            const int r = e >> 4, g = e & 15;
            *reinterpret_cast<float4*>(lvh + r * FU_RS + g * 8) = *reinterpret_cast<const float4*>(a.Vh + r * FU_D + g * 8);
            *reinterpret_cast<float4*>(lvl + r * FU_RS + g * 8) = *reinterpret_cast<const float4*>(a.Vl + r * FU_D + g * 8);
        }
        if (threadIdx.x < 32) {
            const int f = threadIdx.x;
            const bool on = f < a.LK;
            // floor-window coefficients P_f, Q_f (certification below), rounded up
            const double iwu = (double)(1.0f / a.w) * (1.0 + 0x1p-20);      // >= 1/w
            lpn0[f] = on ? (float)((FU_A1H * a.pnorm[f] * (1.0 + 0x1p-20) + FU_A2 * FU_SQRT_D) * iwu * (1.0 + 0x1p-18)) : 0.f;
            lv10[f] = on ? (float)((FU_A2 * a.v1[f] * (1.0 + 0x1p-20) + (0x1p-40 + 0x1p-23) * fabs((double)a.tv[f])) *
                                   iwu * (1.0 + 0x1p-18)) : 0.f;
            lt0[f] = on ? a.tv[f] : 0.f;
            lr0[f] = on ? a.rv[f] : 0;
        }
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 31, h = lane >> 5;
    const float ecf = a.cbound[0], ebf = a.cbound[1], cmaxf = a.cbound[3];
    const bool c_ok = __float_as_uint(a.cbound[2]) == 0u;
    const _Float16* my_h = lch + col * FU_RS + 8 * h;
    const _Float16* my_l = lcl + col * FU_RS + 8 * h;
    const int ntile32 = Kpad >> 5;
    const int64_t ntiles = (a.N + 31) >> 5;
    // LIST: this block's segment of the input list
    const int32_t* lrows = LIST ? a.list_in + (int64_t)blockIdx.x * a.list_seg_rows : nullptr;
    const int64_t lcnt = LIST ? (int64_t)a.list_counts[2 * blockIdx.x] : 0;
    const int64_t ptile0 = LIST ? (int64_t)blockIdx.x * ((a.list_seg_rows + 31) >> 5) : 0;   // part slots

#if WAVE_OFFSET
    // Waves w and w+4 share a SIMD; starting the second half of the block late
    // keeps the two out of phase (one in its MFMA-heavy loop while the other
    // runs VALU-heavy epilogues) instead of lockstep.
    if (wave >= FP_WAVES / 2)
        for (int i = 0; i < WAVE_OFFSET; i++) __builtin_amdgcn_s_sleep(127);
#endif
#if YOUNG_PRIO
    // static priority for the second-dispatched half (MI355X_MICROARCH.md,
    // "Two waves per SIMD", item 4)
    if (wave >= FP_WAVES / 2) __builtin_amdgcn_s_setprio(YOUNG_PRIO);
#endif
    PT_DECL
    const int64_t tbeg = LIST ? wave : (int64_t)blockIdx.x * FP_WAVES + wave;
    const int64_t tend = LIST ? (lcnt + 31) >> 5 : ntiles;
    const int64_t tstep = LIST ? FP_WAVES : (int64_t)gridDim.x * FP_WAVES;
    for (int64_t tile = tbeg; tile < tend; tile += tstep) {
        int64_t row = tile * 32 + col;
        bool valid = row < a.N;
        if (LIST) {
            valid = row < lcnt;
            row = lrows[valid ? row : lcnt - 1];
        }
        const int64_t ptile = ptile0 + tile;      // pass-state slot

        // ---- point -> registers and the split B operand
        float xf[64];
        if constexpr (ROWS != 0) {
            load_row_gen<ROWS>(a, valid ? row : a.N - 1, h, xf);
        } else {
            // rows past N read row N-1 (results for them are never written)
            const float* xr = a.X + (valid ? row : a.N - 1) * FU_D + 8 * h;
#pragma unroll
            for (int s = 0; s < 8; s++) {
                const float4 p0 = *reinterpret_cast<const float4*>(xr + 16 * s);
                const float4 p1 = *reinterpret_cast<const float4*>(xr + 16 * s + 4);
                xf[8 * s + 0] = p0.x; xf[8 * s + 1] = p0.y; xf[8 * s + 2] = p0.z; xf[8 * s + 3] = p0.w;
                xf[8 * s + 4] = p1.x; xf[8 * s + 5] = p1.y; xf[8 * s + 6] = p1.z; xf[8 * s + 7] = p1.w;
            }
        }
        half8 bh[8], bl[8];
        float2v n2a = {0.f, 0.f}, n2b = {0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 8; s++) {
            split8p(xf + 8 * s, bh[s], bl[s]);
#pragma unroll
            for (int j = 0; j < 8; j += 4) {
                const float2v u = {xf[8 * s + j], xf[8 * s + j + 1]}, v = {xf[8 * s + j + 2], xf[8 * s + j + 3]};
                n2a = __builtin_elementwise_fma(u, u, n2a);
                n2b = __builtin_elementwise_fma(v, v, n2b);
            }
        }
        float xn2f = (n2a.x + n2a.y) + (n2b.x + n2b.y);
        xn2f += __shfl_xor(xn2f, 32);
        // f32 sum of squares: inflate by 2^-16 (> d 2^-24) to stay an upper bound;
        // |x|_1 <= sqrt(d) |x|_2 replaces the L1 norm in the A2 terms, and
        // |x|_2 <= 2^15 implies the f16 range guard |x_j| <= 2^15 (false for nan/inf).
        const double xn2 = (double)xn2f * (1.0 + 0x1p-16);
        const double nx = sqrt(xn2);
        const double x1 = FU_SQRT_D * nx;
        const bool x_ok = xn2f <= FU_RANGE * FU_RANGE;

        PT_MARK(0)
        // ---- hash tile + LSH outputs (k = 4: table l = 2g + h lives in registers 4g..4g+3)
        if (HASH) {
            uint32_t fmask = 0;
            // hi products: a fresh MFMA per 16-dim step (<= 15 roundings each),
            // steps added in f32 (+7), then + lo (+1): <= 23 roundings of sum|terms|
            // instead of 128 for one chain (FU_A1H), which cuts the floors left to
            // the fix-up pass ~4x.
            float acc_hi[16];
            {
                const _Float16* vh_row = lvh + col * FU_RS + 8 * h;
                const _Float16* vl_row = lvl + col * FU_RS + 8 * h;
                floatx16 acc_lo, tot;
#pragma unroll
                for (int s = 0; s < 8; s++) {
                    const half8 ah = *reinterpret_cast<const half8*>(vh_row + 16 * s);
                    const half8 al = *reinterpret_cast<const half8*>(vl_row + 16 * s);
                    const floatx16 z = {};
                    const floatx16 acc_s = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], z, 0, 0, 0);
                    acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], s ? acc_lo : z, 0, 0, 0);
                    acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s], acc_lo, 0, 0, 0);
                    if (s == 0) {
                        tot = acc_s;
                    } else {
#pragma unroll
                        for (int r = 0; r < 16; r += 2) {
                            const float2v t2 = {tot[r], tot[r + 1]}, a2 = {acc_s[r], acc_s[r + 1]};
                            const float2v u2 = t2 + a2;
                            tot[r] = u2.x;
                            tot[r + 1] = u2.y;
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < 16; r++) acc_hi[r] = tot[r] + acc_lo[r];
            }
            // Certification in f32 (the floor only needs y to ~2^-20): with
            // u = f32(dot~ + t), y = f32(u * f32(1/w)),
            //   |y - (x.v + t)/w| <= (Ed + 2^-23 |u| + 2^-40 |t|) / w + 2^-21 |y|,
            // Ed = A1 |v||x| + A2 (|v|_1 + |x|_1) + 2^-23 |dot~| (the split bound and
            // the final hi + lo add; the reference's x87 / double-product roundings
            // are below 2^-50 (|v||x| + |t|)). With |x|_1 <= sqrt(d) |x|, |dot~| <=
            // |u| + |t| and |u| / w <= |y| (1 + 2^-19), that is at most
            //   B = |y| G + |x| P_f + Q_f,   G = (2^-22 + 2^-20)(1 + 2^-18),
            //   P_f = (A1 |v| + A2 sqrt(d)) / w,  Q_f = (A2 |v|_1 + (2^-23 + 2^-40)|t|) / w
            // (prologue; the 1 + 2^-18 factors cover the f32 roundings of B, y - B,
            // y + B): floor(y - B) == floor(y + B) certifies the reference's floorl.
            const float iw = 1.0f / a.w;
            const float nxf = (float)nx * (1.f + 0x1p-20f);
            constexpr float G = (0x1p-22f + 0x1p-20f) * (1.f + 0x1p-18f);
            // Opaque zero: keeps the per-function constants as LDS reads inside
            // the loop instead of hoisted VGPRs.
            int hc = 0;
            asm volatile("" : "+v"(hc));
            const float* lt = lt0 + hc;
            const float* lP = lpn0 + hc;
            const float* lQ = lv10 + hc;
            const int32_t* lr = lr0 + hc;
            if (!x_ok && valid) fmask = (a.LK >= 32 ? 0xFFFFFFFFu : (1u << a.LK) - 1u);
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int l = 2 * g + h;
                if (l >= a.L || !valid) continue;
                int32_t hv[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int f = 4 * l + q;
                    const float u = acc_hi[4 * g + q] + lt[f];       // f32(hi + lo sums) + t
                    const float y = u * iw;
                    const float B = fmaf(fabsf(y), G, fmaf(nxf, lP[f], lQ[f]));
                    const float lo = floorf(y - B), hi = floorf(y + B);
                    hv[q] = (int32_t)lo;
                    if (lo != hi) fmask |= 1u << f;   // provisional; redone by hash_fixup_kernel
                }
                const int64_t o = row * a.L + l;
                if (a.tuples) *reinterpret_cast<int4*>(a.tuples + o * 4) = make_int4(hv[0], hv[1], hv[2], hv[3]);
                uint32_t hn = 0;   // flagged values are provisional: the fix-up redoes their table
#pragma unroll
                for (int q = 0; q < 4; q++) hn += phi_term_small(hv[q], lr[4 * l + q]);
                const uint32_t ph = phi_final(hn);
                if (a.phi) a.phi[o] = (int32_t)ph;
                if (a.bucket) a.bucket[o] = bucket_fast(ph, a.bdiv);
            }
            fmask |= __shfl_xor(fmask, 32);
            const unsigned long long fb = __ballot(fmask != 0u && h == 1);
            if (fb) {
                // rows whose floor the split bound cannot certify: (row << 32 | fn mask)
                const int leader = __builtin_ctzll(fb);
                int base = 0;
                if (lane == leader) base = atomicAdd(lcount + 1, __popcll(fb));
                base = __shfl(base, leader);
                if (fmask != 0u && h == 1)
                    hfix_seg[base + __popcll(fb & ((1ull << lane) - 1ull))] = ((unsigned long long)row << 32) | fmask;
            }
        }

        PT_MARK(1)
        // ---- all centroid tiles from the resident image
        // Each score carries its in-tile index (4g+q) in its low 4 mantissa bits:
        // a perturbation below 16 ulp <= 2^-19 |t|, |t| <= |x| cmax + cmax^2/2,
        // charged to E (with 2x margin). The running max then identifies the
        // winner without a compare/select per score; its tile is noted per tile.
        // cosine: |t| <= |x| |c^| (no -|c|^2/2 term); + 2^-43 |x| covers the
        // normalisation's roundings and the reference's own: its q = x.c / (|x||c|)
        // carries <= 2^-46 relative (the fp64 norm chains), and 1 - q rounds at 2^-52
        const float E = MET == 0
            ? (float)(nx * (double)ecf + (double)ebf + FU_A2 * x1 + 0x1p-41 * xn2 +
                      0x1p-18 * (nx * (double)cmaxf + 0.5 * (double)cmaxf * (double)cmaxf) +
                      (ROWS == 2 ? 0x1p-24 * nx * (double)cmaxf : 0.0)) * (1.f + 0x1p-20f) + 1e-30f
            : (float)(nx * (double)ecf + (double)ebf + FU_A2 * x1 + 0x1p-41 * xn2 +
                      0x1p-18 * nx * (double)cmaxf + 0x1p-43 * nx) * (1.f + 0x1p-20f) + 1e-30f;
        float m1 = -__builtin_inff(), m2 = -__builtin_inff();
        int t1 = 0;
        if (MP && !a.pass_first) {
            const float4 st = a.part[ptile * 64 + lane];
            m1 = st.x; m2 = st.y; t1 = __float_as_int(st.z);
        }
        const int tg0 = MP ? a.t0 : 0;        // global index of this slice's first tile
#if PIPE_TILES
        // Software pipeline: tile t's scores are formed (16 VGPRs), then tile
        // t+1's 24 MFMAs issue with tile t's epilogue placed in their gaps
        // (2 VALU per MFMA, well inside the 24 free cycles of each 32-cycle MFMA).
        floatx16 acc_hi, acc_lo;
        tile_mfma(my_h, my_l, bh, bl, acc_hi, acc_lo);
#pragma unroll 1
        for (int t = 0; t < ntile32; t++) {
            float sv[16];
            tile_scores(acc_hi, acc_lo, lcn + t * 32 + 4 * h, sv);
            const float m1_prev = m1;
            if (t + 1 < ntile32) {
                tile_mfma(my_h + (t + 1) * 32 * FU_RS, my_l + (t + 1) * 32 * FU_RS, bh, bl, acc_hi, acc_lo);
                tile_epilogue(sv, m1, m2);
#pragma unroll
                for (int s = 0; s < 8; s++) {
                    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS read: A operands
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // VALU: epilogue
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                }
            } else {
                tile_epilogue(sv, m1, m2);
            }
            t1 = m1 != m1_prev ? t + tg0 : t1;
        }
#else
#if MFMA_PRIO
        __builtin_amdgcn_s_setprio(MFMA_PRIO);
#endif
#pragma unroll TILE_UNROLL
        for (int t = 0; t < ntile32; t++) {
            const float m1_prev = m1;
            float sv[16];
#if ONE_ACC
            floatx16 acc;
            tile_mfma1(my_h + t * 32 * FU_RS, my_l + t * 32 * FU_RS, bh, bl, acc);
            tile_scores1(acc, lcn + t * 32 + 4 * h, sv);
#else
            floatx16 acc_hi, acc_lo;
            tile_mfma(my_h + t * 32 * FU_RS, my_l + t * 32 * FU_RS, bh, bl, acc_hi, acc_lo);
            tile_scores(acc_hi, acc_lo, lcn + t * 32 + 4 * h, sv);
#endif
            tile_epilogue(sv, m1, m2);
            t1 = m1 != m1_prev ? t + tg0 : t1;
        }
#if MFMA_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
#endif
        if (MP && !a.pass_last) {             // more slices to come: carry the state
            a.part[ptile * 64 + lane] = make_float4(m1, m2, __int_as_float(t1), 0.f);
            continue;
        }
        const uint32_t l1 = __float_as_uint(m1) & 0xFu;
        const int i1 = t1 * 32 + 8 * (int)(l1 >> 2) + 4 * h + (int)(l1 & 3u);
        const float om1 = __shfl_xor(m1, 32), om2 = __shfl_xor(m2, 32);
        const int oi1 = __shfl_xor(i1, 32);
        const float M2 = fmaxf(fmaxf(m2, om2), fminf(m1, om1));
        const int I1 = (om1 > m1 || (om1 == m1 && oi1 < i1)) ? oi1 : i1;
        const float M1 = fmaxf(m1, om1);
        const bool cert = x_ok && c_ok && ((double)M2 < (double)M1 - 2.0 * (double)E);

        // ---- winner distance in reference order: the squares are independent,
        // only the sum is a chain; dims 8seg..8seg+7 belong to lane half seg & 1.
        // The exact row is re-read here (L2-resident: this wave loaded it moments
        // ago) rather than held in 64 VGPRs through the MFMA loop.
        // The chain is re-laid for the L1: lane (p, q) = 4 * p + q owns the
        // contiguous quarter dims [32q, 32q+32) of point 16r + p (round r = 0, 1),
        // so each 16-B lane load is a quarter of one 64-B sector of a row (4 lanes
        // fill it) instead of a half-used sector per lane. The row and the winner's
        // fp64 row are re-read from L2; the squares are formed with every lane
        // active, then the quarters add in order, handing the sum on with a quad
        // DPP move.
        PT_MARK(2)
        if constexpr (MET == 1) {
            // cosine winner: one lane per point re-reads its row (L2) and the
            // winner's fp64 row; declined certificates -> the fix-up list
            bool fix = false;
            if (h == 1 && valid && cert) {
                a.assign[row] = I1;
                double v;
                bool okc;
                if constexpr (ROWS == 1) okc = cosine_fast_nb(a.X + row * a.d, a.Cd + (size_t)I1 * a.d, a.d, a.nbv[I1], v);
                else if constexpr (ROWS == 2) okc = cosine_fast_nb(a.X64 + row * a.d, a.Cd + (size_t)I1 * a.d, a.d, a.nbv[I1], v);
                else okc = cosine_fast_nb(a.X + row * FU_D, a.C64 + (size_t)I1 * FU_D, FU_D, a.nbv[I1], v);
                if (okc) a.dist[row] = v;
                else fix = true;
            }
            const unsigned long long fb = __ballot(fix);
            if (fb) {
                const int leader = __builtin_ctzll(fb);
                int base = 0;
                if (lane == leader) base = atomicAdd(lcount + 1, __popcll(fb));
                base = __shfl(base, leader);
                if (fix) hfix_seg[base + __popcll(fb & ((1ull << lane) - 1ull))] = (unsigned long long)row;
            }
        } else {
#if FP_KEEP_X
        {
            // exact row still in registers (B-operand layout): lane half h owns
            // dims 16s+8h..+7; only the winner's fp64 row is loaded
            const double* crow = a.C64 + (size_t)I1 * FU_D + 8 * h;
            double acc = 0.0;
            double2 cbuf[CHAIN_PF][4];
            double2 xnext[4];                 // fp64 rows: the exact values, one step ahead
            const int64_t rowc = valid ? row : a.N - 1;
            if constexpr (ROWS == 2) load_x64_step(a, rowc, 0, h, xnext);
#pragma unroll
            for (int s = 0; s < CHAIN_PF; s++)
#pragma unroll
                for (int j = 0; j < 4; j++) cbuf[s][j] = *reinterpret_cast<const double2*>(crow + 16 * s + 2 * j);
#pragma unroll
            for (int s = 0; s < 8; s++) {
                double sq[8];
                double2 cur[4];
#pragma unroll
                for (int j = 0; j < 4; j++) cur[j] = cbuf[s % CHAIN_PF][j];
                if (s + CHAIN_PF < 8) {
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        cbuf[s % CHAIN_PF][j] = *reinterpret_cast<const double2*>(crow + 16 * (s + CHAIN_PF) + 2 * j);
                }
                double2 xcur[4];
                if constexpr (ROWS == 2) {
#pragma unroll
                    for (int j = 0; j < 4; j++) xcur[j] = xnext[j];
                    if (s + 1 < 8) load_x64_step(a, rowc, s + 1, h, xnext);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++) xcur[j] = make_double2((double)xf[8 * s + 2 * j], (double)xf[8 * s + 2 * j + 1]);
                }
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const double2 cc = cur[j];
                    const double d0 = __dsub_rn(xcur[j].x, cc.x);
                    const double d1 = __dsub_rn(xcur[j].y, cc.y);
                    // LSHKM_DIST_CERTIFIED: x*x (the chain within 2^-44 of the
                    // reference's, inside the 2^-20 contract); exact: glibc's pow
                    sq[2 * j] = a.fast_dist ? __dmul_rn(d0, d0) : gp_sq(d0);
                    sq[2 * j + 1] = a.fast_dist ? __dmul_rn(d1, d1) : gp_sq(d1);
                }
                if (h == 0) {
#pragma unroll
                    for (int j = 0; j < 8; j++) acc = __dadd_rn(acc, sq[j]);
                }
                acc = take_from_lower(acc);
                if (h == 1) {
#pragma unroll
                    for (int j = 0; j < 8; j++) acc = __dadd_rn(acc, sq[j]);
                }
                acc = take_from_upper(acc);
            }
            if (h == 1 && valid && cert) {
                a.assign[row] = I1;
                a.dist[row] = sqrt(acc);
            }
        }
#else
        const int q4 = lane & 3, p4 = lane >> 2;
#pragma unroll 1
        for (int r = 0; r < 2; r++) {
            const int pt = 16 * r + p4;                              // point within the tile
            const int Ip = __shfl(I1, pt);                           // lane pt (half 0) holds it
            const int cp = __shfl((int)cert, pt);
            const int64_t prow = tile * 32 + pt;
            const bool pv = prow < a.N;
            const float* xq = a.X + (pv ? prow : a.N - 1) * FU_D + 32 * q4;
            const double* cq = a.C64 + (size_t)Ip * FU_D + 32 * q4;  // Ip < K always (padding scores are far below)
            double sq[32];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const float4 xv = *reinterpret_cast<const float4*>(xq + 4 * u);
                const double2 c0 = *reinterpret_cast<const double2*>(cq + 4 * u);
                const double2 c1 = *reinterpret_cast<const double2*>(cq + 4 * u + 2);
                const double d0 = __dsub_rn((double)xv.x, c0.x), d1 = __dsub_rn((double)xv.y, c0.y);
                const double d2 = __dsub_rn((double)xv.z, c1.x), d3 = __dsub_rn((double)xv.w, c1.y);
                sq[4 * u] = gp_sq(d0);
                sq[4 * u + 1] = gp_sq(d1);
                sq[4 * u + 2] = gp_sq(d2);
                sq[4 * u + 3] = gp_sq(d3);
            }
            double acc = 0.0;
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                if (q4 == qq) {
#pragma unroll
                    for (int j = 0; j < 32; j++) acc = __dadd_rn(acc, sq[j]);
                }
                if (qq < 3) {
                    const double moved = quad_shift_up(acc);         // lane q takes lane q-1's sum
                    if (q4 == qq + 1) acc = moved;
                }
            }
            if (q4 == 3 && pv && cp) {
                a.assign[prow] = Ip;
                a.dist[prow] = sqrt(acc);
            }
        }
#endif
        }
        PT_MARK(3)
        const bool amb = valid && !cert;
        const unsigned long long amask = __ballot(amb && h == 1);
        if (h == 1 && valid) {
            if (!cert) {
                int base = 0;
                const int leader = __builtin_ctzll(amask);
                if (lane == leader) base = atomicAdd(lcount, __popcll(amask));
                base = __shfl(base, leader);
                const int rank = __popcll(amask & ((1ull << lane) - 1ull));
                ambig_seg[base + rank] = (int32_t)row;
            }
        }
        PT_MARK(4)
    }
    PT_FLUSH
    __syncthreads();
    // slot 0: ambiguous rows (the last pass decides them); slot 1: the hash
    // fix-up list (the hashing pass) or the cosine fix-up list (the last pass)
    if (threadIdx.x < 2 && (!MP || (threadIdx.x == 0 ? a.pass_last != 0 : (HASH || (MET == 1 && a.pass_last))))) {
        const int c = lcount[threadIdx.x];
        a.seg_counts[2 * blockIdx.x + threadIdx.x] = c;
        if (c) atomicAdd(threadIdx.x == 0 ? a.ambig_count : a.hfix_count, (unsigned long long)c);
    }
}

// ------------------------------------------------------------ hi-only form
// Lloyd (+ hashing, euclidean) with ONE f16 MFMA per centroid product: the
// score is t~ = acc(-|c|^2/2 + sum_j xh_j ch_j), the accumulator initialised
// with the f32 -|c|^2/2 (no epilogue add), ch = f16(f32(c)), xh = f16(x);
// cosine (MET = 1): the normalised centroid rows, no offset.
// Bound (rigorous, |x_j| <= 2^15, c in range): with xr = x - xh (exact in f32)
// and cr = c - ch,
//   |t~ - t| <= |xh||cr| + |xr||c| + 2^-24|cn| + A (|cn| + |xh||ch|),
//   A = 130 2^-23 (<= 129 round-toward-zero additions of partial sums bounded
//   by |cn| + sum|xh_j ch_j|), plus the terms of the 3-product form for the
//   reference's own fp64 roundings (2^-41 (|x|^2 + |c|^2)) and the packed tile
//   index (2^-18 (|x||c| + |cn|)); |xr| is summed per row, the centroid
//   maxima come from the prep (cbound[3..6]). A point is certified iff
//   M2 < M1 - 2E; the others (~3% of N(0,1) rows at K = 256) are listed for the
//   3-product form (fused_persistent_kernel<..., LIST>), which certifies all but
//   ~1% of those and lists the rest for the exact pass.
// One third of the MFMA work of the 3-product form, and only the hi image of
// the centroids in LDS: up to 512 centroids per pass (K = 1024: 2 passes).
constexpr int FH_KMAX = 512;
__host__ __device__ constexpr int fh_lds_bytes(int Kpad, bool hash) {
    return 16 + Kpad * FU_RS * 2 + Kpad * 4 + (hash ? 2 * 32 * FU_RS * 2 + FP_HC_BYTES : 0);
}
static_assert(fh_lds_bytes(FH_KMAX, true) <= 160 * 1024, "hi-only LDS image exceeds 160 KiB");
constexpr double FH_A = 130.0 * 0x1p-23;

// Waves per block of the hi-only form (one block per CU), per instantiation.
// Measured for the single-pass euclidean hash form (fused pass, N = 10M, K =
// 256): 8 waves 2.37 ms; 12 waves (~30 spilled loop invariants) 2.74 ms; 12
// waves with the row re-read for the chain instead of kept (one lane per row
// over two tiles) 3.7 ms -- the lane-per-row re-reads of the row and of the
// winner's fp64 row thrash L1. K = 1024 (two passes, both without spills at
// 12 waves): first pass (hash) 1.91 -> 1.88 ms at 12 waves, second pass
// (chain) 2.48 -> 2.59 ms -- a third wave per SIMD does not pay. FH_WAVES_SET
// forces one count for all (experiments).
#ifndef FH_WAVES_MPFAST
#define FH_WAVES_MPFAST 12     // the last pass of the multi-pass form with the certified distance
#endif
template <bool HASH, bool MP, int MET, bool FAST = false>
#ifndef FH_FAST_WAVES
#define FH_FAST_WAVES 8     // the single-pass FAST form (the headline kernel)
#endif
__host__ __device__ constexpr int fh_waves() {
#ifdef FH_WAVES_SET
    return FH_WAVES_SET;
#else
    return HASH && MP ? 12 : (MP && FAST ? FH_WAVES_MPFAST : (FAST && !MP ? FH_FAST_WAVES : 8));
#endif
}
constexpr int FH_WAVES_MIN = 8, FH_WAVES_MAX = 12;

// The upper half's finish of the cosine winner certificate (IpAcc, exact.h):
// the halves' double-double sums joined by one TwoSum; sum_k |S_k| bound
// rounded up (+ 2^-47 relative for the roundings of |A_k + B_end| and of the
// sums here; the partial sums stand in for the exact ones: their TwoSum rests,
// |sl| <= 64 2^-53 max|t| per half, and the offsets, <= 2^-38 max|t|, charged
// absolutely -- a cancelling A_k + B_end must not hide them). max |t| of both
// halves' running sums <= sum_j |p_j| <= (1 + 2^-53) |x| |c| (Cauchy-Schwarz):
// mb = 2 sqrt(xa nbv) (1 + 2^-40) bounds the pair of them without a per-term
// max; sum |S_k| >= 2^-790 stands in for quot_status's lower range check on
// the partial sums themselves (max |S_k| >= that / 128).
__device__ inline int cosine_halves_finish(double sh0, double sl0, double ts0, double sh, double sl, double ts,
                                           double xa, double nbv, double& v) {
    const double mb = 2.0 * sqrt(__dmul_rn(xa, nbv)) * (1.0 + 0x1p-40);
    const double tsum = __dadd_rn(ts0, ts);
    if (!(tsum >= 0x1p-790)) return 2;
    IpAcc ip;
    const double t = __dadd_rn(sh0, sh);
    const double bb = __dsub_rn(t, sh0);
    const double e = __dadd_rn(__dsub_rn(sh0, __dsub_rn(t, bb)), __dsub_rn(sh, bb));
    ip.sh = t;
    ip.sl = __dadd_rn(__dadd_rn(sl0, sl), e);
    ip.ts = __dadd_rn(tsum * (1.0 + 0x1p-47), 0x1p-37 * mb);
    ip.mx = mb;
    double q, qr;
    const int st = ip.quot_status(__dmul_rn(sqrt(xa), sqrt(nbv)), q, qr);
    if (st == 0) v = __dsub_rn(1.0, q);
    return st;
}

// MET = 1: cosine (the prep's normalised centroid rows, score x.c^ with no
// offset; the winner's distance from the row in registers, declines to the
// cfix list). HASH with MET = 1: CosineHGen signs of the L*k projections
// (k = 4: table l = 2g + h in D registers 4g..4g+3), certified as in
// hash_mfma.hip, g = phi = bucket; uncertified signs to the hfix list.
// Cosine winner distance from the row in registers, both lane halves busy.
// Lane half h owns dims 16s + 8h..+7 (s = 0..7). Each half accumulates the
// double products of ITS dims with IpAcc's double-double (exact.h), in its own
// order; the reference's x87 chain runs over all 128 in order (block 2s = half
// 0's step s, block 2s + 1 = half 1's), so its partial sums are S_k = A_k +
// B_end(s-1) in half 0's block s and S_k = B_k + A_end(s) in half 1's. The
// halves trade their running sums after every step: half 0 adds |A_k + B_end(s-1)|
// exactly as the reference's partial sum, half 1 |B_k + A_end(s-1)| plus
// 8 |A_end(s) - A_end(s-1)| (the block it runs one step behind) -- the round-4
// bound 8 (sum |A_end| + sum |B_end|) roughly doubled sum_k |S_k| and declined
// 9.3 % of the C3 winners. max |S_k| from the norms (cosine_halves_finish;
// exact.h quot_status decides). |x|^2 is the reference's sequential chain, the
// halves taking turns (the euclidean winner's pattern).
// Returns 0 (certified, v = 1 - q), 1 / 2 (declined: soft-x87 fix-up).
__device__ inline int cosine_winner_halves(const float (&xf)[64], const double* __restrict__ crow_h, double nbv, int h,
                                           double& v) {
    // |x|^2: the reference's sequential fp64 chain (cust_vector.hpp:139-155), halves alternating
    double xa = 0.0;
#pragma unroll
    for (int s = 0; s < 8; s++) {
        if (h == 0) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const double xj = (double)xf[8 * s + j];
                xa = __dadd_rn(xa, __dmul_rn(xj, xj));
            }
        }
        xa = take_from_lower(xa);
        if (h == 1) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const double xj = (double)xf[8 * s + j];
                xa = __dadd_rn(xa, __dmul_rn(xj, xj));
            }
        }
        xa = take_from_upper(xa);
    }
    // the inner product, each half over its own dims
    double sh = 0.0, sl = 0.0, ts = 0.0;
    double off = 0.0;                     // half 0: B_end(s-1); half 1: A_end(s-1)
    double2 cb[4];
#pragma unroll
    for (int j = 0; j < 4; j++) cb[j] = *reinterpret_cast<const double2*>(crow_h + 2 * j);
#pragma unroll
    for (int s = 0; s < 8; s++) {
        double cv[8];
#pragma unroll
        for (int j = 0; j < 4; j++) { cv[2 * j] = cb[j].x; cv[2 * j + 1] = cb[j].y; }
        if (s + 1 < 8) {
#pragma unroll
            for (int j = 0; j < 4; j++) cb[j] = *reinterpret_cast<const double2*>(crow_h + 16 * (s + 1) + 2 * j);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const double pj = __dmul_rn((double)xf[8 * s + j], cv[j]);
            const double t = __dadd_rn(sh, pj);
            const double bb = __dsub_rn(t, sh);
            const double e = __dadd_rn(__dsub_rn(sh, __dsub_rn(t, bb)), __dsub_rn(pj, bb));   // TwoSum
            sh = t;
            sl = __dadd_rn(sl, e);
            ts = __dadd_rn(ts, fabs(__dadd_rn(t, off)));
        }
        // trade the running sums: half 0 takes B_end(s), half 1 A_end(s) (and
        // charges the block it ran behind: 8 |A_end(s) - A_end(s-1)|)
        const double other = swap_halves(sh, h);
        if (h == 1) ts = __dadd_rn(ts, 8.0 * fabs(__dsub_rn(other, off)));
        off = other;
    }
    // the lower half's accumulator to the upper lanes
    const double sh0 = swap_halves(sh, h), sl0 = swap_halves(sl, h), ts0 = swap_halves(ts, h);
    if (h == 0) return 2;                 // the upper lanes finish
    return cosine_halves_finish(sh0, sl0, ts0, sh, sl, ts, xa, nbv, v);
}

// The same for fp64 rows (ROWS = 2): the exact x values re-read from the row
// (L2) two 16-dim steps ahead (a rolled loop: unrolled, the loads of all steps
// were hoisted and spilled) for the halves' inner products. Dims past d are
// zero in the row (load_x64_step) and in the padded centroid copy: exact zero
// terms. |x|^2 of a general double row needs glibc's pow(x, 2) per term
// (gpow2.h): the row's sequential sum comes precomputed (a.xn2, row_sumsq).
__device__ inline int cosine_winner_halves_x64(const FusedArgs& a, int64_t rowc, const double* __restrict__ crow_h,
                                               double nbv, int h, double& v) {
    double2 xn[4], xnn[4];
    load_x64_step(a, rowc, 0, h, xn);
    load_x64_step(a, rowc, 1, h, xnn);
    double sh = 0.0, sl = 0.0, ts = 0.0;
    double off = 0.0;                     // as cosine_winner_halves
    double2 cb[4];
#pragma unroll
    for (int j = 0; j < 4; j++) cb[j] = *reinterpret_cast<const double2*>(crow_h + 2 * j);
#pragma unroll 1
    for (int s = 0; s < 8; s++) {
        double xv[8], cv[8];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            xv[2 * j] = xn[j].x; xv[2 * j + 1] = xn[j].y;
            cv[2 * j] = cb[j].x; cv[2 * j + 1] = cb[j].y;
            xn[j] = xnn[j];
        }
        if (s + 2 < 8) load_x64_step(a, rowc, s + 2, h, xnn);
        if (s + 1 < 8) {
#pragma unroll
            for (int j = 0; j < 4; j++) cb[j] = *reinterpret_cast<const double2*>(crow_h + 16 * (s + 1) + 2 * j);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const double pj = __dmul_rn(xv[j], cv[j]);
            const double t = __dadd_rn(sh, pj);
            const double bb = __dsub_rn(t, sh);
            const double e = __dadd_rn(__dsub_rn(sh, __dsub_rn(t, bb)), __dsub_rn(pj, bb));   // TwoSum
            sh = t;
            sl = __dadd_rn(sl, e);
            ts = __dadd_rn(ts, fabs(__dadd_rn(t, off)));
        }
        const double other = swap_halves(sh, h);
        if (h == 1) ts = __dadd_rn(ts, 8.0 * fabs(__dsub_rn(other, off)));
        off = other;
    }
    const double sh0 = swap_halves(sh, h), sl0 = swap_halves(sl, h), ts0 = swap_halves(ts, h);
    if (h == 0) return 2;
    return cosine_halves_finish(sh0, sl0, ts0, sh, sl, ts, a.xn2[rowc], nbv, v);
}

// NIMG = 2 (512 < K <= 1024, euclidean): ONE launch for all centroids. The
// LDS holds one 512-centroid image at a time; the block's waves each score
// their tile against the image in LDS, the block swaps in the other image
// (two barriers, 128 KB from L2), and the waves finish the same tile against
// it with the row still in registers -- no second read of X and no carried
// pass state. Images alternate A,B / B,A between rounds (one swap per round);
// every wave runs the block's round count (tiles past the end: no valid rows).
// GATH (euclidean, one pass, Kpad <= FH_GATH_KMAX): the winner rows of the
// distance chain are gathered into a per-wave LDS ring by LDS-DMA, 8 lanes per
// 128-B row segment (coalesced), instead of 16-B register loads from 32
// different rows per instruction -- the vector-memory path (TA/TD/TCP) was the
// busiest unit of the pass (TD 97 %, TA 88 % busy; 63 % of the L1 accesses
// were these loads). Ring of two 4-KiB steps (16 dims x 32 points x 8 B).
constexpr int FH_GATH_STEP = 32 * 16 * 8;
constexpr int FH_GATH_WAVE = 2 * FH_GATH_STEP;
constexpr int FH_GATH_KMAX = 256;
__host__ __device__ constexpr int fh_gath_off(int Kpad, bool hash) { return (fh_lds_bytes(Kpad, hash) + 255) & ~255; }
static_assert(fh_gath_off(FH_GATH_KMAX, true) + 8 * FH_GATH_WAVE <= 160 * 1024, "gather ring exceeds 160 KiB");

// One LDS-DMA piece: each lane's 16 B at gsrc land at lds_dst + 16 * lane
// (M0 written and restored in the same statement; the load is invisible to the
// compiler's wait counting: the chain waits for it with an explicit vmcnt).
__device__ inline void glds16(const void* gsrc, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

// ROWS = 0: fp32 rows of 128 dims (X); 1: fp32 rows of d <= 128 dims; 2: fp64
// rows of d <= 128 dims (X64) -- euclidean Lloyd without hashing, one pass.
// Dims d..127 are zero in the row and in the centroid images (the prep pads
// them). fp64 rows: the scores use xh = f16(f32(x)); |x - f32(x)| <= 2^-24 |x|
// joins |xr| in the bound; the winner chain re-reads the fp64 row (the
// register copy is f32).
// FAST (euclidean, fp32 rows; the last pass when K > 512): the certified f32 winner distance
// compiled in (no fp64 chain state). Its f32 centroid rows are register loads:
// through the gather ring (GATH) each 16-dim step waits on its DMA, and the
// short f32 sum cannot hide that (fused pass 2.21 vs 2.14 ms at C3).
template <bool HASH, bool MP = false, int MET = 0, int NIMG = 1, bool GATH = false, int ROWS = 0, bool FAST = false>
__global__ __launch_bounds__((64 * fh_waves<HASH, MP, MET, FAST>()), 1) void fused_hi_kernel(FusedArgs a) {
    constexpr int FH_WAVES = fh_waves<HASH, MP, MET, FAST>();
    constexpr int FH_THREADS = 64 * FH_WAVES;
    static_assert(NIMG == 1 || (!MP && MET == 0), "two-image form: euclidean, single launch");
    static_assert(!GATH || (!MP && MET == 0 && NIMG == 1 && FH_WAVES == 8), "gather ring: euclidean single pass");
    static_assert(ROWS == 0 || (!HASH && !MP && NIMG == 1), "general rows: Lloyd without hashing, one pass");
    // the gather's explicit vmcnt waits assume no other vector loads in the chain
    static_assert(!(GATH && ROWS == 2), "fp64 rows re-read x in the chain: register loads of the winner rows");
    static_assert(!FAST || (MET == 0 && ROWS != 2 && NIMG == 1 && !GATH), "fast distance: euclidean, fp32 rows");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int Kpad = a.Kpad;
    const bool fastd = FAST || a.fast_dist != 0;
    const int KI = NIMG == 2 ? FH_KMAX : Kpad;           // centroid rows the LDS image holds
    int* lcount = reinterpret_cast<int*>(smem);          // [0] uncertified rows, [1] hash fix-up rows, [2] cosine declines
    _Float16* lch = reinterpret_cast<_Float16*>(smem + 16);
    float* lcn = reinterpret_cast<float*>(lch + KI * FU_RS);
    _Float16* lvh = reinterpret_cast<_Float16*>(lcn + KI);
    _Float16* lvl = lvh + 32 * FU_RS;
    float* lpn0 = reinterpret_cast<float*>(lvl + 32 * FU_RS);
    float* lv10 = lpn0 + 32;
    float* lt0 = lv10 + 32;
    int32_t* lr0 = reinterpret_cast<int32_t*>(lt0 + 32);

    // image img: centroid rows [img * KI, img * KI + rows) into LDS rows 0..
    auto load_image = [&](int img) {
        const int r0 = img * KI, nr = NIMG == 2 && img == 1 ? Kpad - FH_KMAX : KI;
        // FH_CU granules per thread in flight at once (a plain copy loop waited on every load)
        constexpr int FH_CU = 8;
        for (int e0 = 0; e0 < nr * 16; e0 += FH_THREADS * FH_CU) {
            float4 v[FH_CU];
#pragma unroll
            for (int u = 0; u < FH_CU; u++) {
                // past the end: granule 0 again (the same bytes rewritten), so neither
                // the loads nor the stores carry a branch and the loads issue together
                const int e = e0 + u * FH_THREADS + (int)threadIdx.x < nr * 16 ? e0 + u * FH_THREADS + (int)threadIdx.x : 0;
                v[u] = *reinterpret_cast<const float4*>(a.Ch + (size_t)(r0 + (e >> 4)) * FU_D + (e & 15) * 8);
            }
#pragma unroll
            for (int u = 0; u < FH_CU; u++) {
                const int e = e0 + u * FH_THREADS + (int)threadIdx.x < nr * 16 ? e0 + u * FH_THREADS + (int)threadIdx.x : 0;
                *reinterpret_cast<float4*>(lch + (e >> 4) * FU_RS + (e & 15) * 8) = v[u];
            }
        }
        for (int e = threadIdx.x; e < nr; e += FH_THREADS) lcn[e] = a.cnh[r0 + e];
    };
    load_image(0);
    if (threadIdx.x < 3) lcount[threadIdx.x] = 0;
    int32_t* ambig_seg = a.ambig + (int64_t)blockIdx.x * a.seg_rows;
    unsigned long long* hfix_seg = a.hfix + (int64_t)blockIdx.x * a.seg_rows;
    unsigned long long* cfix_seg = a.cfix ? a.cfix + (int64_t)blockIdx.x * a.seg_rows : nullptr;
    if (HASH) {
        for (int e = threadIdx.x; e < 32 * 16; e += FH_THREADS) {
            const int r = e >> 4, g = e & 15;
            *reinterpret_cast<float4*>(lvh + r * FU_RS + g * 8) = *reinterpret_cast<const float4*>(a.Vh + r * FU_D + g * 8);
            *reinterpret_cast<float4*>(lvl + r * FU_RS + g * 8) = *reinterpret_cast<const float4*>(a.Vl + r * FU_D + g * 8);
        }
        if (threadIdx.x < 32) {
            const int f = threadIdx.x;
            const bool on = f < a.LK;
            // euclidean: the window in units of y = (acc + t) / w; cosine: of the
            // inner product itself (hash_mfma.hip)
            const double iwu = MET == 1 ? 1.0 : (double)(1.0f / a.w) * (1.0 + 0x1p-20);
            const double tf = MET == 1 || !on ? 0.0 : fabs((double)a.tv[f]);
            lpn0[f] = on ? (float)((FU_A1H * a.pnorm[f] * (1.0 + 0x1p-20) + FU_A2 * FU_SQRT_D) * iwu * (1.0 + 0x1p-18)) : 0.f;
            lv10[f] = on ? (float)((FU_A2 * a.v1[f] * (1.0 + 0x1p-20) + (0x1p-40 + 0x1p-23) * tf) * iwu * (1.0 + 0x1p-18) +
                                   0x1p-126) : 0.f;
            lt0[f] = on && MET == 0 ? a.tv[f] : 0.f;
            lr0[f] = on && MET == 0 ? a.rv[f] : 0;
        }
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 31, h = lane >> 5;
    const float cmaxf = a.cbound[3], crf = a.cbound[4], chf = a.cbound[5], cnf = a.cbound[6];
    const bool c_ok = __float_as_uint(a.cbound[2]) == 0u;
    const _Float16* my_h = lch + col * FU_RS + 8 * h;
    const int ntile32 = Kpad >> 5;
    const int64_t ntiles = (a.N + 31) >> 5;
    // point-independent part of the bound
    const double Ec = (0x1p-24 + FH_A) * (double)cnf + 0x1p-41 * (double)cmaxf * (double)cmaxf + 0x1p-18 * (double)cnf;

    const int64_t tstride = (int64_t)gridDim.x * FH_WAVES, tfirst = (int64_t)blockIdx.x * FH_WAVES;
    const int64_t nround = NIMG == 2 && ntiles > tfirst ? (ntiles - tfirst + tstride - 1) / tstride : 0;
    int64_t rd = 0;
    // profiling build: [0] row load + split + hash tile, [1] centroid tiles, [2] certificate + winner chain + stores
    // this lane's 64 values of row (tile, col) in the B-operand layout (rows past
    // the end read row N-1: their results are never stored)
    auto load_row = [&](int64_t tl, float (&dst)[64]) {
        if constexpr (ROWS != 0) {
            const int64_t rr = tl * 32 + col;
            load_row_gen<ROWS>(a, rr < a.N ? rr : a.N - 1, h, dst);
            return;
        }
        const int64_t rr = tl * 32 + col;
        const float* xr = a.X + (rr < a.N ? rr : a.N - 1) * FU_D + 8 * h;
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const float4 p0 = *reinterpret_cast<const float4*>(xr + 16 * s);
            const float4 p1 = *reinterpret_cast<const float4*>(xr + 16 * s + 4);
            dst[8 * s + 0] = p0.x; dst[8 * s + 1] = p0.y; dst[8 * s + 2] = p0.z; dst[8 * s + 3] = p0.w;
            dst[8 * s + 4] = p1.x; dst[8 * s + 5] = p1.y; dst[8 * s + 6] = p1.z; dst[8 * s + 7] = p1.w;
        }
    };
    // XPF: the next tile's row is loaded while this tile's winner chain waits on
    // its fp64 centroid rows (the HBM latency hides behind the L2 round trips)
    constexpr bool xpf = XPF && NIMG == 1;
    float xf[64];
    if (xpf && tfirst + wave < ntiles) load_row(tfirst + wave, xf);
    PT_DECL
    for (int64_t tile = tfirst + wave; NIMG == 2 ? rd < nround : tile < ntiles; tile += tstride, rd++) {
        const int64_t row = tile * 32 + col;
        const bool valid = row < a.N;
        if (!xpf) load_row(tile, xf);
        half8 bh[8];
        float2v n2a = {0.f, 0.f}, n2b = {0.f, 0.f}, r2 = {0.f, 0.f};
        // hi part of 8 values (LO: and the lo part), |x|^2 and |x - xh|^2 partial sums
        auto split_step = [&](int s, half8& lo, auto lo_tag) {
            split8_hi<decltype(lo_tag)::value>(xf + 8 * s, bh[s], lo, r2);
#pragma unroll
            for (int j = 0; j < 8; j += 4) {
                const float2v u = {xf[8 * s + j], xf[8 * s + j + 1]}, v = {xf[8 * s + j + 2], xf[8 * s + j + 3]};
                n2a = __builtin_elementwise_fma(u, u, n2a);
                n2b = __builtin_elementwise_fma(v, v, n2b);
            }
        };
        double xn2, nx, nxr, nxh;
        bool x_ok;
        auto finish_norms = [&]() {
            float xn2f = (n2a.x + n2a.y) + (n2b.x + n2b.y);
            float xr2f = r2.x + r2.y;
            xn2f += __shfl_xor(xn2f, 32);
            xr2f += __shfl_xor(xr2f, 32);
            // f32 sums of squares inflated by 2^-16 (> d 2^-24): upper bounds
            xn2 = (double)xn2f * (1.0 + 0x1p-16);
            nx = sqrt(xn2);
            nxr = sqrt((double)xr2f * (1.0 + 0x1p-16)) + 0x1p-100;
            if (ROWS == 2) nxr += 0x1p-24 * nx * (1.0 + 0x1p-20);   // |x - f32(x)| (fp64 rows)
            nxh = nx + nxr;                                     // |xh| <= |x| + |xr|
            x_ok = xn2f <= FU_RANGE * FU_RANGE;
        };
        const bool hash_here = HASH;          // <HASH, MP>: the first pass only
        if (!hash_here) {
#pragma unroll
            for (int s = 0; s < 8; s++) {
                half8 unused;
                split_step(s, unused, std::false_type{});
            }
            finish_norms();
        }

        if (hash_here) {
            uint32_t fmask = 0;
            float acc_hi[16];
            {
                const _Float16* vh_row = lvh + col * FU_RS + 8 * h;
                const _Float16* vl_row = lvl + col * FU_RS + 8 * h;
                // per 16-dim step: the lo products first, then the hi products into
                // the same accumulator (16 roundings relative to the step's sum of
                // |terms|, the lo parts' own roundings ~2^-11 smaller), steps added
                // in f32 (+7): 23 -> 24 roundings, still inside FU_A1H; one
                // accumulator fewer than the separate lo chain (fits 168 VGPRs)
                floatx16 tot;
#pragma unroll
                for (int s = 0; s < 8; s++) {
                    half8 bls;
                    split_step(s, bls, std::true_type{});
                    const half8 ah = *reinterpret_cast<const half8*>(vh_row + 16 * s);
                    const half8 al = *reinterpret_cast<const half8*>(vl_row + 16 * s);
                    const floatx16 z = {};
                    floatx16 acc_s = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s], z, 0, 0, 0);
                    acc_s = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bls, acc_s, 0, 0, 0);
                    acc_s = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc_s, 0, 0, 0);
                    if (s == 0) {
                        tot = acc_s;
                    } else {
#pragma unroll
                        for (int r = 0; r < 16; r += 2) {
                            const float2v t2 = {tot[r], tot[r + 1]}, a2 = {acc_s[r], acc_s[r + 1]};
                            const float2v u2 = t2 + a2;
                            tot[r] = u2.x;
                            tot[r + 1] = u2.y;
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < 16; r++) acc_hi[r] = tot[r];
            }
            finish_norms();
            // the floor certificate of fused_persistent_kernel (same bound)
            const float iw = MET == 1 ? 1.f : 1.0f / a.w;
            const float nxf = (float)nx * (1.f + 0x1p-20f);
            constexpr float G = (0x1p-22f + 0x1p-20f) * (1.f + 0x1p-18f);
            int hc = 0;
            asm volatile("" : "+v"(hc));
            const float* lt = lt0 + hc;
            const float* lP = lpn0 + hc;
            const float* lQ = lv10 + hc;
            const int32_t* lr = lr0 + hc;
            if (!x_ok && valid) fmask = (a.LK >= 32 ? 0xFFFFFFFFu : (1u << a.LK) - 1u);
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int l = 2 * g + h;
                if (l >= a.L || !valid) continue;
                const int64_t o = row * a.L + l;
                if constexpr (MET == 1) {
                    // CosineHGen: ip >= 0, certified when |acc~| exceeds the window;
                    // CosineGGen: g = bits MSB first
                    int gv = 0;
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int f = 4 * l + q;
                        const float u = acc_hi[4 * g + q];
                        const float B = fmaf(nxf, lP[f], lQ[f]);
                        gv = (gv << 1) | (u >= 0.f ? 1 : 0);
                        if (!(fabsf(u) > B)) fmask |= 1u << f;
                    }
                    if (a.phi) a.phi[o] = gv;
                    if (a.bucket) a.bucket[o] = gv;
                    continue;
                }
                int32_t hv[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int f = 4 * l + q;
                    const float u = acc_hi[4 * g + q] + lt[f];
                    const float y = u * iw;
                    const float B = fmaf(fabsf(y), G, fmaf(nxf, lP[f], lQ[f]));
                    const float lo = floorf(y - B), hi = floorf(y + B);
                    hv[q] = (int32_t)lo;
                    if (lo != hi) fmask |= 1u << f;
                }
                if (a.tuples) *reinterpret_cast<int4*>(a.tuples + o * 4) = make_int4(hv[0], hv[1], hv[2], hv[3]);
                uint32_t hn = 0;
#pragma unroll
                for (int q = 0; q < 4; q++) hn += phi_term_small(hv[q], lr[4 * l + q]);
                const uint32_t ph = phi_final(hn);
                if (a.phi) a.phi[o] = (int32_t)ph;
                if (a.bucket) a.bucket[o] = bucket_fast(ph, a.bdiv);
            }
            fmask |= __shfl_xor(fmask, 32);
            const unsigned long long fb = __ballot(fmask != 0u && h == 1);
            if (fb) {
                const int leader = __builtin_ctzll(fb);
                int base = 0;
                if (lane == leader) base = atomicAdd(lcount + 1, __popcll(fb));
                base = __shfl(base, leader);
                if (fmask != 0u && h == 1)
                    hfix_seg[base + __popcll(fb & ((1ull << lane) - 1ull))] = ((unsigned long long)row << 32) | fmask;
            }
        }

        PT_MARK(0)
        // the certificate's bound E depends on the row only: formed before the
        // centroid tiles (its fp64 ops overlap the MFMAs). cosine: + 2^-43 |x| for the normalisation and the reference's own q
        // (fused_persistent_kernel's cosine bound)
        const double E = (nxh * (double)crf + nxr * (double)cmaxf + FH_A * nxh * (double)chf + 0x1p-41 * xn2 +
                          0x1p-18 * nx * (double)cmaxf + (MET == 1 ? 0x1p-43 * nx : 0.0) + Ec) * (1.0 + 0x1p-20) +
                         1e-30;
        // ---- centroid tiles: 8 MFMAs each, accumulator initialised with -|c|^2/2
        float m1 = -__builtin_inff(), m2 = -__builtin_inff();
        int t1 = 0;
        if (MP && !HASH && !a.pass_first) {
            const float4 st = a.part[tile * 64 + lane];
            m1 = st.x; m2 = st.y; t1 = __float_as_int(st.z);
        }
        const int tg0 = MP ? a.t0 : 0;
#if MFMA_PRIO
        __builtin_amdgcn_s_setprio(MFMA_PRIO);
#endif
        const int ntile_run = ntile32;
        auto run_tiles = [&](int ntl, int tgo) {
#pragma unroll TILE_UNROLL
            for (int t = 0; t < ntl; t++) {
                const float m1_prev = m1;
                floatx16 acc;
                const float* cn_t = lcn + t * 32 + 4 * h;     // D rows 8g + 4h + q of registers 4g + q
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const float4 cn = *reinterpret_cast<const float4*>(cn_t + 8 * g);
                    acc[4 * g] = cn.x; acc[4 * g + 1] = cn.y; acc[4 * g + 2] = cn.z; acc[4 * g + 3] = cn.w;
                }
                const _Float16* arow = my_h + t * 32 * FU_RS;
#pragma unroll
                for (int s = 0; s < 8; s++) {
                    const half8 ah = *reinterpret_cast<const half8*>(arow + 16 * s);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc, 0, 0, 0);
                }
                float sv[16];
#pragma unroll
                for (int r = 0; r < 16; r++) sv[r] = acc[r];
                tile_epilogue(sv, m1, m2);
                t1 = m1 != m1_prev ? t + tgo : t1;
            }
        };
        if (NIMG == 1) {
            run_tiles(ntile_run, tg0);
        } else {
            // the image in LDS at this round's start, then the other one
            const int i0 = (int)(rd & 1);
            const int nA = FH_KMAX / 32, nB = (Kpad - FH_KMAX) / 32;
            run_tiles(i0 == 0 ? nA : nB, i0 * nA);
            __syncthreads();
            load_image(1 - i0);
            __syncthreads();
            run_tiles(i0 == 0 ? nB : nA, (1 - i0) * nA);
        }
#if MFMA_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        PT_MARK(1)
        float xn[64];
        if (xpf && tile + tstride < ntiles) load_row(tile + tstride, xn);
        // <HASH, MP> launches only the first of several passes (never the last)
        if (MP && (HASH || !a.pass_last)) {
            a.part[tile * 64 + lane] = make_float4(m1, m2, __int_as_float(t1), 0.f);
            if (xpf) {
#pragma unroll
                for (int j = 0; j < 64; j++) xf[j] = xn[j];
            }
            continue;
        }
        const uint32_t l1 = __float_as_uint(m1) & 0xFu;
        const int i1 = t1 * 32 + 8 * (int)(l1 >> 2) + 4 * h + (int)(l1 & 3u);
        const float om1 = __shfl_xor(m1, 32), om2 = __shfl_xor(m2, 32);
        const int oi1 = __shfl_xor(i1, 32);
        const float M2 = fmaxf(fmaxf(m2, om2), fminf(m1, om1));
        const int I1 = (om1 > m1 || (om1 == m1 && oi1 < i1)) ? oi1 : i1;
        const float M1 = fmaxf(m1, om1);
        // the winner's fp64 row: the first loads go out before the certificate
        // and the list append
        const double* crow = a.C64 + (size_t)I1 * FU_D + 8 * h;
        // GATH: piece u of a step holds points 8u..8u+7, lane L the 16-B chunk
        // (L & 7) ^ swz(p) of point p = 8u + (L >> 3) (swz(p) = (p >> 1) & 7: the
        // lanes of each ds_read_b128 group hit 16 distinct 4-bank groups).
        // g32 (every centroid value is an f32, e.g. dataset rows: the prep's
        // cbound[7] == 0): the f32 image C32 instead, exact as doubles -- half the
        // bytes and two pieces per step: piece u holds points 16u..16u+15, lane L
        // the 16-B chunk (L & 3) ^ swz32(p) of point p = 16u + (L >> 2), swz32(p) =
        // (p >> 2) & 3 (the 16 lanes of a ds_read_b128 group on distinct banks).
        const char* gsrc[4];
        uint32_t gbase = 0;
        const bool g32 = GATH && a.C32 != nullptr && (__float_as_uint(a.cbound[7]) & 1u) == 0u;
        const int gstep = g32 ? 64 : 128;                // bytes of one 16-dim step of a row
        if (GATH && !fastd) {
            gbase = (uint32_t)__builtin_amdgcn_readfirstlane(
                (int)((uint32_t)(uintptr_t)(smem + fh_gath_off(Kpad, HASH)) + (uint32_t)wave * FH_GATH_WAVE));
            if (g32) {
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const int p = 16 * u + (lane >> 2);
                    const int Ip = __shfl(I1, p);
                    gsrc[u] = reinterpret_cast<const char*>(a.C32 + (size_t)Ip * FU_D + 4 * ((lane & 3) ^ ((p >> 2) & 3)));
                }
                gsrc[2] = gsrc[3] = gsrc[0];
#pragma unroll
                for (int s0 = 0; s0 < 2; s0++)
#pragma unroll
                    for (int u = 0; u < 2; u++) glds16(gsrc[u] + gstep * s0, gbase + s0 * FH_GATH_STEP + u * 1024);
            } else {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int p = 8 * u + (lane >> 3);
                    const int Ip = __shfl(I1, p);
                    gsrc[u] = reinterpret_cast<const char*>(a.C64 + (size_t)Ip * FU_D + 2 * ((lane & 7) ^ ((p >> 1) & 7)));
                }
#pragma unroll
                for (int s0 = 0; s0 < 2; s0++)
#pragma unroll
                    for (int u = 0; u < 4; u++) glds16(gsrc[u] + gstep * s0, gbase + s0 * FH_GATH_STEP + u * 1024);
            }
        }
        // GATH: a step's values come from the ring one step early (the LDS read
        // overlaps the previous step's chain), the ring slot is refilled two
        // steps ahead as soon as it is read
        double2 gnext[4];
        float4 gnext32[2];                    // g32: raw f32 chunks, widened when used
        auto gread = [&](int st) {
            const char* ring = smem + fh_gath_off(Kpad, HASH) + wave * FH_GATH_WAVE + (st & 1) * FH_GATH_STEP;
            if (g32) {
#pragma unroll
                for (int j = 0; j < 2; j++)
                    gnext32[j] = *reinterpret_cast<const float4*>(ring + (col >> 4) * 1024 + (col & 15) * 64 +
                                                                  16 * ((2 * h + j) ^ ((col >> 2) & 3)));
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    gnext[j] = *reinterpret_cast<const double2*>(ring + col * 128 + 16 * ((4 * h + j) ^ ((col >> 1) & 7)));
            }
        };
        // vmcnt(n): all but the wave's n youngest vector-memory operations done
        // (one step's pieces: 2 for g32, else 4)
        auto wait_step = [&]() {
            if (g32) __builtin_amdgcn_s_waitcnt(0x0F72);                   // vmcnt(2)
            else __builtin_amdgcn_s_waitcnt(0x0F74);                       // vmcnt(4)
        };
        // ring step s consumed: slot s & 1 refilled with step s + 2, step s + 1 read
        auto ring_advance = [&](int s) {
            if (s + 2 < 8) {
                __builtin_amdgcn_s_waitcnt(0xC07F);                        // lgkmcnt(0): slot s & 1 is read
                asm volatile("" ::: "memory");
                if (g32) {
#pragma unroll
                    for (int u = 0; u < 2; u++) glds16(gsrc[u] + gstep * (s + 2), gbase + (s & 1) * FH_GATH_STEP + u * 1024);
                } else {
#pragma unroll
                    for (int u = 0; u < 4; u++) glds16(gsrc[u] + gstep * (s + 2), gbase + (s & 1) * FH_GATH_STEP + u * 1024);
                }
            }
            if (s + 1 < 8) {
                if (s + 2 < 8) wait_step();                                // step s + 1 landed
                else __builtin_amdgcn_s_waitcnt(0x0F70);                    // vmcnt(0)
                asm volatile("" ::: "memory");
                gread(s + 1);
            }
        };
        // fp64 rows: the chain's x values re-read (mostly L2) four 16-dim steps
        // ahead (one step ahead left the chain waiting ~8 round trips per tile)
        constexpr int XD = 4;
        double2 xring[XD][4];
        const int64_t rowc = row < a.N ? row : a.N - 1;
        if constexpr (ROWS == 2 && MET == 0) {
#pragma unroll
            for (int st = 0; st < XD; st++) load_x64_step(a, rowc, st, h, xring[st]);
        }
        double2 cbuf[CHAIN_PF][4];
        if (MET == 0 && !GATH && !fastd) {
#pragma unroll
            for (int s = 0; s < CHAIN_PF; s++)
#pragma unroll
                for (int j = 0; j < 4; j++) cbuf[s][j] = CHAIN_LD(crow + 16 * s + 2 * j, 8 * s + 2 * j);
        }
        const bool cert = x_ok && c_ok && ((double)M2 < (double)M1 - 2.0 * E);

        // euclidean fast distance (fastd): the winner's distance from f32(c)
        // in f32 with every lane busy, certified to 2^-20 relative (DESIGN.md §5:
        // 8 accumulators per lane, <= 12 roundings per sum, plus the f32(c)
        // residual |c - f32(c)| of the centroid); a row whose bound fails is
        // refined like an uncertified argmin (the exact chain of the LIST form)
        bool dok = true;
        double fdist = 0.0;
        if constexpr (MET == 0) {
            if (fastd) {
                const float* c32 = a.C32 + (size_t)I1 * FU_D + 8 * h;
                float2v q[4] = {};
#pragma unroll
                for (int s = 0; s < 8; s++) {
                    const float4 c0 = *reinterpret_cast<const float4*>(c32 + 16 * s);
                    const float4 c1 = *reinterpret_cast<const float4*>(c32 + 16 * s + 4);
                    const float2v cv[4] = {{c0.x, c0.y}, {c0.z, c0.w}, {c1.x, c1.y}, {c1.z, c1.w}};
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const float2v xv = {xf[8 * s + 2 * j], xf[8 * s + 2 * j + 1]};
                        const float2v dv = xv - cv[j];
                        q[j] = __builtin_elementwise_fma(dv, dv, q[j]);
                    }
                }
                float t = ((q[0].x + q[0].y) + (q[1].x + q[1].y)) + ((q[2].x + q[2].y) + (q[3].x + q[3].y));
                t = t + swap_halves_f(t, h);
                const double S = (double)t, R = (double)a.rn32[I1];
                const double B = 14.2 * 0x1p-24 * S + 2.02 * R * sqrt(S) + 2.02 * R * R + 0x1p-100;
                dok = B <= 0x1p-19 * S;                   // false for inf / nan
                fdist = sqrt(S);
            }
        }
        const bool amb = valid && !(cert && dok);
        const unsigned long long amask = __ballot(amb && h == 1);
        if (amb && h == 1) {
            int base = 0;
            const int leader = __builtin_ctzll(amask);
            if (lane == leader) base = atomicAdd(lcount, __popcll(amask));
            base = __shfl(base, leader);
            ambig_seg[base + __popcll(amask & ((1ull << lane) - 1ull))] = (int32_t)row;
        }
        if constexpr (MET == 1) {
            // cosine winner from the row in registers, both lane halves busy;
            // declined certificates -> the fix-up list
            bool fix = false;
            if (valid && cert) {                          // the same on both halves of a point
                double v = 0.0;
                int st;
                // fp32 rows (ROWS = 0 / 1): the values in registers are exact (zero
                // past d, as the padded centroid copy); fp64 rows re-read
                if constexpr (ROWS == 2) st = cosine_winner_halves_x64(a, row, a.C64 + (size_t)I1 * FU_D + 8 * h, a.nbv[I1], h, v);
                else st = cosine_winner_halves(xf, a.C64 + (size_t)I1 * FU_D + 8 * h, a.nbv[I1], h, v);
                if (h == 1) {
                    a.assign[row] = I1;
                    if (st == 0) a.dist[row] = v;
                    else fix = true;
                }
            }
            const unsigned long long fb = __ballot(fix);
            if (fb) {
                const int leader = __builtin_ctzll(fb);
                int base = 0;
                if (lane == leader) base = atomicAdd(lcount + 2, __popcll(fb));
                base = __shfl(base, leader);
                if (fix) cfix_seg[base + __popcll(fb & ((1ull << lane) - 1ull))] = (unsigned long long)row;
            }
        } else if (fastd) {
            if (h == 1 && valid && cert && dok) {
                a.assign[row] = I1;
                a.dist[row] = fdist;
            }
        } else {
        {
            // winner distance in reference order from the row kept in registers:
            // the lane halves take turns on the chain, 8 dims each
#if CHAIN_PRIO
            __builtin_amdgcn_s_setprio(CHAIN_PRIO);
#endif
            double acc = 0.0;
            PwAcc pw;
            // fp64 rows: glibc's pow in the chain itself when the launch gave the
            // LDS for it (gp_sq_wave; every difference of general doubles has
            // more than 26 bits, so the PwAcc test would list every row)
            double* pwl = nullptr;
            if constexpr (ROWS == 2) {
                if (a.pw_lds) pwl = reinterpret_cast<double*>(smem + a.pw_lds) + wave * 512;
            }
            if constexpr (GATH) {
                wait_step();                                               // step 0 landed
                asm volatile("" ::: "memory");
                gread(0);
            }
#pragma unroll
            for (int s = 0; s < 8; s++) {
                double sq[8];
                double2 cur[4];
                if constexpr (GATH) {
                    if (g32) {
#pragma unroll
                        for (int j = 0; j < 2; j++) {
                            cur[2 * j] = make_double2((double)gnext32[j].x, (double)gnext32[j].y);
                            cur[2 * j + 1] = make_double2((double)gnext32[j].z, (double)gnext32[j].w);
                        }
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; j++) cur[j] = gnext[j];
                    }
                    ring_advance(s);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++) cur[j] = cbuf[s % CHAIN_PF][j];
                    if (s + CHAIN_PF < 8) {
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            cbuf[s % CHAIN_PF][j] = CHAIN_LD(crow + 16 * (s + CHAIN_PF) + 2 * j, 8 * (s + CHAIN_PF) + 2 * j);
                    }
                }
                double2 xcur[4];
                if constexpr (ROWS == 2) {
#pragma unroll
                    for (int j = 0; j < 4; j++) xcur[j] = xring[s % XD][j];
                    if (s + XD < 8) load_x64_step(a, rowc, s + XD, h, xring[s % XD]);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++) xcur[j] = make_double2((double)xf[8 * s + 2 * j], (double)xf[8 * s + 2 * j + 1]);
                }
                double dv[8];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const double2 cc = cur[j];
                    dv[2 * j] = __dsub_rn(xcur[j].x, cc.x);
                    dv[2 * j + 1] = __dsub_rn(xcur[j].y, cc.y);
                }
                if (ROWS == 2 && pwl) {
                    gp_sq_wave<8>(dv, sq, pwl);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        sq[j] = __dmul_rn(dv[j], dv[j]);
                        // the reference squares with glibc pow: x*x is its value when
                        // the square is exact; otherwise the row's distance is redone
                        // by the fix-up (gpow2.h PwAcc: differences of <= 26 bits, and
                        // for fp64 rows no tiny ones)
                        pw.add<ROWS == 2>(dv[j]);
                    }
                }
                if (h == 0) {
#pragma unroll
                    for (int j = 0; j < 8; j++) acc = __dadd_rn(acc, sq[j]);
                }
                acc = take_from_lower(acc);
                if (h == 1) {
#pragma unroll
                    for (int j = 0; j < 8; j++) acc = __dadd_rn(acc, sq[j]);
                }
                acc = take_from_upper(acc);
            }
            // fp32 rows: a difference 0 < |x - c| < 2^-460 needs such a centroid
            // value (x has >= 2^-149 magnitude or is zero), flagged by the prep
            const bool pw_hard = pwl == nullptr && (pw.hard() || (ROWS != 2 && (__float_as_uint(a.cbound[7]) & 2u) != 0u));
            // the shuffle outside the ||: evaluated only where pw_hard is false, it
            // would read the other half's lane while that lane is masked off
            const int pw_other = __shfl_xor((int)pw_hard, 32);
            const bool hard = pw_hard || pw_other != 0;
            if (h == 1 && valid && cert) {
                a.assign[row] = I1;
                if (!hard) a.dist[row] = sqrt(acc);
            }
            // the pow fix-up list (cfix, counts in slot 2): certified winners
            // whose chain met an inexact square
            const unsigned long long pb = __ballot(h == 1 && valid && cert && hard);
            if (pb) {
                const int leader = __builtin_ctzll(pb);
                int base = 0;
                if (lane == leader) base = atomicAdd(lcount + 2, __popcll(pb));
                base = __shfl(base, leader);
                if (h == 1 && valid && cert && hard) cfix_seg[base + __popcll(pb & ((1ull << lane) - 1ull))] = (unsigned long long)row;
            }
#if CHAIN_PRIO
            __builtin_amdgcn_s_setprio(0);
#endif
        }
        }
        PT_MARK(2)
        if (xpf) {
#pragma unroll
            for (int j = 0; j < 64; j++) xf[j] = xn[j];
        }
    }
    PT_FLUSH
    __syncthreads();
    if (threadIdx.x < 2 && (!MP || (threadIdx.x == 0 ? (!HASH && a.pass_last != 0) : (HASH && a.pass_first)))) {
        const int c = lcount[threadIdx.x];
        a.seg_counts[2 * blockIdx.x + threadIdx.x] = c;
        if (c) atomicAdd(threadIdx.x == 0 ? a.ambig_count : a.hfix_count, (unsigned long long)c);
    }
    // slot 2: cosine declines / euclidean pow fix-ups (exact distances)
    if ((MET == 1 || !fastd) && threadIdx.x == 2 && (!MP || (!HASH && a.pass_last))) {
        const int c = lcount[2];
        a.cfix_counts[2 * blockIdx.x + 1] = c;
        if (c) atomicAdd(a.cfix_count, (unsigned long long)c);
    }
}

// Rows listed by the fused pass with an uncertified floor (euclidean) or sign
// (cosine): fix-up pass. Four lanes per listed row, each holding 32 contiguous
// dims and 8 of the row's tuples (or 2 of its g values); the next row of the
// group is loaded while the current one is computed, and the projections and
// per-function constants sit in LDS, so the only global latency per row is
// the prefetched one. The fp64 products are summed per lane and then across the
// 4 lanes: hash.hip's bound covers any summation order of the 128 products
// (depth 34 < 130); the soft-x87 fallback keeps the reference order.
constexpr int HF_WAVES = 4;
#ifndef HF_SPLIT_SET
#define HF_SPLIT_SET 4
#endif
constexpr int HF_SPLIT = HF_SPLIT_SET;                // blocks per list segment
constexpr int HF_G = 4;                               // lanes per listed row
constexpr int HF_SLOTS = 64 * HF_WAVES / HF_G;        // rows per block pass
// LDS image of the projections (fp64): dim r at (r / 32) * HF_QS + (r % 32) *
// HF_PS; the quarters skewed by 8 words so that the 4 lanes of a row, reading
// dim 32q + j of the same function, hit different banks (LK <= 32)
constexpr int HF_PS = 33;
constexpr int HF_QS = 32 * HF_PS + 8;
constexpr size_t HF_LDS = (size_t)4 * HF_QS * 8 + 32 * (8 + 8 + 4);
__device__ inline int hf_pidx(int r) { return (r >> 5) * HF_QS + (r & 31) * HF_PS; }

// lane ^ 1 / lane ^ 2 within each quad by DPP quad_perm (VALU moves)
template <int CTRL>
__device__ inline uint32_t quad_swap(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ inline double quad_swap(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint64_t lo = quad_swap<CTRL>((uint32_t)b), hi = quad_swap<CTRL>((uint32_t)(b >> 32));
    return __longlong_as_double((long long)((hi << 32) | lo));
}
constexpr int QP_X1 = 0xB1, QP_X2 = 0x4E;   // quad_perm [1,0,3,2], [2,3,0,1]
// sum over the 4 lanes of a row group (a quad, all active together); every
// lane gets the same value ((v0 + v1) + (v2 + v3) in any lane's operand order)
__device__ inline double group4_sum(double v) {
    v += quad_swap<QP_X1>(v);
    v += quad_swap<QP_X2>(v);
    return v;
}
__device__ inline uint32_t group4_sum(uint32_t v) {
    v += quad_swap<QP_X1>(v);
    v += quad_swap<QP_X2>(v);
    return v;
}

// the rare sequential fallbacks, out of line (their registers would lower the
// occupancy of the whole kernel)
__device__ __noinline__ int32_t fixup_floor_x87(const float* xrow, const double* pts, int f, double tt, float w) {
    sx80 sxs = sx_zero();
    for (int j = 0; j < FU_D; j++) sxs = sx_add_double(sxs, __dmul_rn(pts[hf_pidx(j) + f], (double)xrow[j]));
    sxs = sx_add_double(sxs, tt);
    return (int32_t)sx_floor_i64(sx_div(sxs, sx_from_float(w)));
}
__device__ __noinline__ int fixup_sign_x87(const float* xrow, const double* pts, int f) {
    SxSum sx;
    sx.init();
    for (int j = 0; j < FU_D; j++) sx.add(__dmul_rn(pts[hf_pidx(j) + f], (double)xrow[j]));
    return sx_hash_sign(sx);
}

// One listed row as the group's lane q holds it.
struct FixRow {
    int64_t row;
    uint32_t mask;
    float x[32];       // dims [32q, 32q + 32)
    int32_t v[8];      // euclidean: tuples [8q, 8q + 8); cosine: g of tables 2q, 2q + 1
};

template <bool COS>
__device__ inline void fix_load(const FusedArgs& a, unsigned long long ent, int q, FixRow& r) {
    r.row = (int64_t)(ent >> 32);
    r.mask = (uint32_t)ent;
    const float* xq = a.X + r.row * FU_D + 32 * q;
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const float4 v = *reinterpret_cast<const float4*>(xq + 4 * u);
        r.x[4 * u] = v.x; r.x[4 * u + 1] = v.y; r.x[4 * u + 2] = v.z; r.x[4 * u + 3] = v.w;
    }
    // unconditional loads (clamped indices; the extra values are never used):
    // a load under a branch makes the compiler wait for it at the merge
    if (COS) {
        const int32_t* g = (a.bucket ? a.bucket : a.phi) + r.row * a.L;
#pragma unroll
        for (int i = 0; i < 2; i++) r.v[i] = g[min(2 * q + i, a.L - 1)];
    } else {
        const int32_t* t = a.tuples + r.row * a.LK;
#pragma unroll
        for (int i = 0; i < 8; i++) r.v[i] = t[min(8 * q + i, a.LK - 1)];
    }
}

template <bool COS>
__device__ inline void fix_row(const FusedArgs& a, const double* pts, const double* cpn, const double* ctt,
                               const int32_t* crv, int q, FixRow& r) {
    // four independent accumulators per lane (the fp64 FMA chains of 32 left the
    // waves issue-stalled on their dependencies, 39 % of their cycles): nx only
    // bounds, and the dot product's bound covers any summation order (depth 12 here)
    double xq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 32; j++) xq[j & 3] = fma((double)r.x[j], (double)r.x[j], xq[j & 3]);
    const double nx = sqrt(group4_sum((xq[0] + xq[1]) + (xq[2] + xq[3])));
    const float* xrow = a.X + r.row * FU_D;
    const int k = a.k;
    const double iwd = 1.0 / (double)a.w;
    for (uint32_t m = r.mask; m; m &= m - 1) {
        const int f = __builtin_ctz(m);
        const double* pq = pts + q * HF_QS + f;
        // keep the fp64 widening inside the loop (hoisted, it holds 64 VGPRs)
#pragma unroll
        for (int j = 0; j < 32; j++) asm volatile("" : "+v"(r.x[j]));
        double aq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < 32; j++) aq[j & 3] = fma(pq[j * HF_PS], (double)r.x[j], aq[j & 3]);
        const double acc = group4_sum((aq[0] + aq[1]) + (aq[2] + aq[3]));
        const double P = cpn[f] * nx * (1.0 + 0x1p-40);
        if (COS) {
            const double B = (double)(FU_D + 3) * 0x1p-52 * P + 0x1p-1000;
            int bit;
            if (acc > B && acc < 0x1p1000) bit = 1;
            else if (acc < -B && acc > -0x1p1000) bit = 0;
            else {                                   // the same decision in all 4 lanes
                bit = fixup_sign_x87(xrow, pts, f);
                if (q == 0) atomicAdd(a.stats + STAT_HASH_EXACT, 1ull);
            }
            // g = bits MSB first (CosineGGen): function l*k + i is bit k-1-i of table l
            const int l = f / k, b = 1 << (k - 1 - (f - l * k));
#pragma unroll
            for (int i = 0; i < 2; i++)
                if (l == 2 * q + i) r.v[i] = bit ? (r.v[i] | b) : (r.v[i] & ~b);
        } else {
            // y by the reciprocal (iw = RN(1/w)): three roundings of 2^-53 each
            // relative, inside the |y| 2^-50 term
            const double tt = ctt[f], iw = iwd;
            const double y = (acc + tt) * iw;
            const double B = ((double)(FU_D + 2) * 0x1p-52 * (P + fabs(tt))) * (iw * (1.0 + 0x1p-50)) +
                             fabs(y) * 0x1p-50;
            const double lo = floor(y - B), hi = floor(y + B);
            int32_t hv = (int32_t)lo;
            if (lo != hi) {                          // the same decision in all 4 lanes
                hv = fixup_floor_x87(xrow, pts, f, tt, a.w);
                if (q == 0) atomicAdd(a.stats + STAT_HASH_EXACT, 1ull);
            }
#pragma unroll
            for (int i = 0; i < 8; i++) r.v[i] = f == 8 * q + i ? hv : r.v[i];
            if ((f >> 3) == q) a.tuples[r.row * a.LK + f] = hv;
        }
    }
    const uint32_t kmask = k >= 32 ? 0xFFFFFFFFu : ((1u << k) - 1u);
    if (COS) {
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int l = 2 * q + i;
            if (l < a.L && (r.mask & (kmask << (l * k)))) {
                if (a.phi) a.phi[r.row * a.L + l] = r.v[i];
                if (a.bucket) a.bucket[r.row * a.L + l] = r.v[i];
            }
        }
        return;
    }
    // touched tables: phi from the lanes' partial sums of the phi terms (the
    // uint32 sum wraps the same in any order)
    uint32_t term[8];
#pragma unroll
    for (int i = 0; i < 8; i++) term[i] = 8 * q + i < a.LK ? phi_term(r.v[i], crv[8 * q + i]) : 0u;
    for (int l = 0; l < a.L; l++) {
        if (!(r.mask & (kmask << (l * k)))) continue;                // the same in all 4 lanes
        uint32_t hn = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int f = 8 * q + i;
            hn += f >= l * k && f < l * k + k ? term[i] : 0u;
        }
        hn = group4_sum(hn);
        if (q == 0) {
            const uint32_t ph = phi_final(hn);
            if (a.phi) a.phi[r.row * a.L + l] = (int32_t)ph;
            if (a.bucket) a.bucket[r.row * a.L + l] = bucket_fast(ph, a.bdiv);
        }
    }
}

template <bool COS>
__global__ __launch_bounds__(64 * HF_WAVES) void hash_fixup_kernel(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* pts = reinterpret_cast<double*>(smem);   // skewed [128][32]
    double* cpn = pts + 4 * HF_QS;                   // [32] |p_f| (rounded up)
    double* ctt = cpn + 32;                          // [32] t_f
    int32_t* crv = reinterpret_cast<int32_t*>(ctt + 32);   // [32] r_f
    const int nseg = gridDim.x / HF_SPLIT;       // segments across XCDs (cos_fix_seg_kernel)
    const int seg = blockIdx.x % nseg, part = blockIdx.x / nseg;
    const int n = a.seg_counts[2 * seg + 1];
    if (n == 0) return;                                                 // block-uniform
    const unsigned long long* list = a.hfix + (int64_t)seg * a.seg_rows;
    const int LK = a.LK, LKpad = a.LKpad;
#pragma unroll
    for (int e = threadIdx.x; e < FU_D * 32; e += 64 * HF_WAVES) {
        const int r = e >> 5, f = e & 31;
        pts[hf_pidx(r) + f] = f < LK ? a.PT[r * LKpad + f] : 0.0;
    }
    if (threadIdx.x < 32) {
        const int f = threadIdx.x;
        cpn[f] = f < LK ? a.pnorm[f] : 0.0;
        ctt[f] = !COS && f < LK ? (double)a.tv[f] : 0.0;
        crv[f] = !COS && f < LK ? a.rv[f] : 0;
    }
    __syncthreads();
    const int q = threadIdx.x & (HF_G - 1), slot = threadIdx.x / HF_G;
    constexpr int STRIDE = HF_SPLIT * HF_SLOTS;
    int e = part * HF_SLOTS + slot;
    if (e >= n) return;                                                 // whole groups
    // software pipeline: the next row (and the list entry after it) load while
    // the current one is computed; past the end the last entry is re-loaded
    FixRow cur, nxt;
    fix_load<COS>(a, list[e], q, cur);
    unsigned long long ent2 = list[min(e + STRIDE, n - 1)];
    for (; e < n; e += STRIDE) {
        fix_load<COS>(a, ent2, q, nxt);
        ent2 = list[min(e + 2 * STRIDE, n - 1)];
        fix_row<COS>(a, pts, cpn, ctt, crv, q, cur);
        cur = nxt;
    }
}

// ------------------------------------------------------------------ preparation
// Centroids -> f16 hi/lo rows, -||c||^2/2, and the per-call bound maxima.
constexpr int FP_PREP_WAVES = 8;     // centroids per prep block (Kpad % 64 == 0)
// d < 128: the rows are zero-padded to 128 dims (C64p: the padded fp64 copy the
// winner chains read; a zero dim adds (0 - 0)^2 = +0 to a non-negative chain).
__global__ void fused_centroid_prep(const double* __restrict__ C, int K, int Kpad, _Float16* __restrict__ Ch,
                                    _Float16* __restrict__ Cl, float* __restrict__ cnh, unsigned int* __restrict__ cb,
                                    int metric, double* __restrict__ nbv, float* __restrict__ C32,
                                    float* __restrict__ rn32, int d, double* __restrict__ C64p) {
    const int c = blockIdx.x * FP_PREP_WAVES + (threadIdx.x >> 6);   // one wave per centroid row
    const int lane = threadIdx.x & 63;
    double s2 = 0.0, s1 = 0.0;
    bool bad = false;
    double scale = 1.0;                  // cosine: the row is normalised (score x.c/|c|)
    if (metric == 1) {
        double q = 0.0;
        for (int j = lane; j < FU_D; j += 64) {
            const double v = c < K && j < d ? C[(size_t)c * d + j] : 0.0;
            q = fma(v, v, q);
        }
        for (int off = 32; off >= 1; off >>= 1) q += __shfl_xor(q, off);
        // zero / extreme-norm centroids (the reference's NaN for a zero vector,
        // assignment.hpp:66) leave the call uncertified: every row goes exact
        if (c < K && !(q >= 1e-200 && q <= 1e200)) bad = true;
        scale = (q >= 1e-200 && q <= 1e200) ? 1.0 / sqrt(q) : 0.0;
        if (lane == 0 && c < K) {
            double b = 0.0;
            for (int j = 0; j < d; j++) {
                const double cj = C[(size_t)c * d + j];
                b = __dadd_rn(b, gp_sq(cj));
            }
            nbv[c] = b;
        }
    }
    bool not32 = false;                  // some value of the row is not an f32 (cbound[7] bit 0)
    bool tiny = false;                   // some 0 < |c_j| < 2^-460 (cbound[7] bit 1: PwAcc)
    double rr = 0.0, hh = 0.0;           // |c - ch|^2, |ch|^2 (the hi-only scores' bound)
    double r32 = 0.0;                    // |c - f32(c)|^2 (fast distances)
    for (int j = lane; j < FU_D; j += 64) {
        const double raw = c < K && j < d ? C[(size_t)c * d + j] : 0.0;
        const double v = raw * scale;
        if (C64p) C64p[(size_t)c * FU_D + j] = raw;
        const float f = (float)v;
        not32 |= c < K && (double)f != v;
        tiny |= c < K && fabs(raw) < 0x1p-460 && raw != 0.0;
        if (C32) {
            C32[(size_t)c * FU_D + j] = f;
            const double e = v - (double)f;       // exact (or inf / nan: never certified)
            r32 = fma(e, e, r32);
        }
        const _Float16 hv = (_Float16)f;
        Ch[(size_t)c * FU_D + j] = hv;
        Cl[(size_t)c * FU_D + j] = (_Float16)(f - (float)hv);
        s2 = fma(v, v, s2);
        s1 += fabs(v);
        const double r = v - (double)hv;     // exact in fp64 for |v| <= 2^15
        rr = fma(r, r, rr);
        hh = fma((double)hv, (double)hv, hh);
        bad |= !(fabs(v) <= (double)FU_RANGE);
    }
    for (int off = 32; off >= 1; off >>= 1) {
        s2 += __shfl_xor(s2, off);
        s1 += __shfl_xor(s1, off);
        rr += __shfl_xor(rr, off);
        hh += __shfl_xor(hh, off);
        r32 += __shfl_xor(r32, off);
    }
    // sum of 128 non-negative fp64 values: <= 2^-46 relative rounding; rounded up
    if (rn32 && lane == 0) rn32[c] = r32 == 0.0 ? 0.f : (float)(sqrt(r32) * (1.0 + 0x1p-40)) * (1.f + 0x1p-22f);
    const unsigned long long anybad = __ballot(bad);
    const unsigned long long any_not32 = __ballot(not32);
    const unsigned long long any_tiny = __ballot(tiny);
    // per wave (centroid) the bound maxima, then one atomic per word per block:
    // single-word atomics from every centroid serialise (~12 ns each)
    __shared__ unsigned int wmax[FP_PREP_WAVES][8];
    if (lane == 0) {
        unsigned int m[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        m[7] = (any_not32 ? 1u : 0u) | (any_tiny ? 2u : 0u);
        if (c >= K) {
            // padding rows: a finite score far below any real one (|x.c| < 2^38 under
            // the range guard), so the packed-index trick never meets an inf/nan
            cnh[c] = -0x1p100f;
        } else {
            cnh[c] = metric == 1 ? 0.f : (float)(-0.5 * s2);
            const double up = 1.0 + 0x1p-18;
            const double nc = sqrt(s2) * (1.0 + 0x1p-30);
            // |t~ - t| <= (A1 + 2^-22)|x||c| + A2(|x|_1 + |c|_1) + 2^-23 |c|^2 + 2^-41 (|x|^2 + |c|^2)
            // (cosine: no |c|^2 term in t, c = the normalised row)
            m[0] = __float_as_uint((float)((FU_A1 + 0x1p-22) * nc * up));     // positive floats order like their bits
            m[1] = __float_as_uint((float)((FU_A2 * s1 * (1.0 + 0x1p-20) + (metric == 1 ? 0.0 : 0x1p-23 * s2) +
                                            0x1p-41 * s2) * up));
            m[2] = anybad ? 1u : 0u;
            m[3] = __float_as_uint((float)(nc * up));                        // max |c|, rounded up
            // hi-only scores (fused_hi_kernel): max |c - ch|, max |ch|, max |cn|, rounded up
            m[4] = __float_as_uint((float)(sqrt(rr) * (1.0 + 0x1p-30) * up));
            m[5] = __float_as_uint((float)(sqrt(hh) * (1.0 + 0x1p-30) * up));
            m[6] = __float_as_uint((float)(metric == 1 ? 0.0 : 0.5 * s2 * up));
        }
#pragma unroll
        for (int i = 0; i < 8; i++) wmax[threadIdx.x >> 6][i] = m[i];
    }
    __syncthreads();
    if (threadIdx.x < 8) {
        const int i = threadIdx.x;
        unsigned int v = 0u;
        for (int w = 0; w < FP_PREP_WAVES; w++) v = i == 2 || i == 7 ? (v | wmax[w][i]) : max(v, wmax[w][i]);
        if (v) {
            if (i == 2 || i == 7) atomicOr(cb + i, v);
            else atomicMax(cb + i, v);
        }
    }
}

int launch_fused_prep(hipStream_t s, const double* C, int K, int Kpad, _Float16* Ch, _Float16* Cl, float* cnh,
                      float* cbound, int metric, double* nbv, float* C32, float* rn32, int d, double* C64p) {
    if (d < 1 || d > FU_D || (d != FU_D && metric == 0 && !C64p)) {
        set_error("launch_fused_prep: d <= 128, and d < 128 needs the padded centroid copy");
        return -1;
    }
    if (metric == 1 && !nbv) {
        set_error("launch_fused_prep: cosine needs the norm array");
        return -1;
    }
    if ((C32 == nullptr) != (rn32 == nullptr)) {
        set_error("launch_fused_prep: the fast-distance image needs both arrays");
        return -1;
    }
    (void)hipMemsetAsync(cbound, 0, 32, s);
    if (Kpad % FP_PREP_WAVES) {
        set_error("launch_fused_prep: Kpad must be a multiple of 8");
        return -1;
    }
    hipLaunchKernelGGL(fused_centroid_prep, dim3((unsigned)(Kpad / FP_PREP_WAVES)), dim3(64 * FP_PREP_WAVES), 0, s, C, K, Kpad, Ch, Cl, cnh,
                       reinterpret_cast<unsigned int*>(cbound), metric, nbv, C32, rn32, d, C64p);
    return kstatus("fused_centroid_prep");
}

int launch_fused(hipStream_t s, bool hash, FusedLaunch& f) {
    f.nseg = 0;
    f.side_timed = false;
    if (f.N <= 0) return 0;
    FusedArgs a;
    a.pw_lds = 0;
    a.X = f.X; a.N = f.N;
    a.Ch = f.Ch; a.Cl = f.Cl; a.cnh = f.cnh; a.cbound = f.cbound; a.C64 = f.C64; a.Kpad = f.Kpad;
    a.Vh = f.Vh; a.Vl = f.Vl; a.PT = f.PT; a.tv = f.tv; a.pnorm = f.pnorm; a.v1 = f.v1; a.rv = f.rv;
    a.w = f.w; a.L = f.L; a.k = f.k; a.LK = f.LK; a.LKpad = f.LKpad; a.nb = f.nb;
    a.tuples = f.tuples; a.phi = f.phi; a.bucket = f.bucket; a.assign = f.assign; a.dist = f.dist;
    a.ambig = f.ambig; a.ambig_count = f.ambig_count; a.stats = f.stats;
    a.hfix = f.hfix; a.hfix_count = f.hfix_count;
    a.cfix = f.cfix; a.cfix_counts = f.cfix_counts; a.cfix_count = f.cfix_count;
    a.bdiv = make_bucket_div(f.nb);
    a.nbv = f.nbv;
    a.part = nullptr; a.t0 = 0; a.pass_first = 1; a.pass_last = 1;
    a.prof = nullptr;
    a.C32 = f.C32; a.rn32 = f.rn32;
    a.fast_dist = f.fast_dist && f.metric == 0 && f.rows != 2 && f.C32 && f.rn32 ? 1 : 0;
    a.X64 = f.X64; a.d = f.rows == 0 ? FU_D : f.d; a.xn2 = f.xn2;
    a.xvec = f.rows == 1 ? (f.d % 4 == 0 && ((uintptr_t)f.X & 15) == 0)
                         : (f.d % 2 == 0 && ((uintptr_t)f.X64 & 15) == 0);
    a.Cd = f.Cd;
    if (f.rows != 0 && (hash || !f.hi || f.Kpad > FH_KMAX || f.d < 1 || f.d > FU_D || (f.metric == 1 && !f.Cd) ||
                        (f.rows == 1 ? !f.X : (f.rows != 2 || !f.X64)))) {
        set_error("launch_fused: general rows run the hi-only form without hashing, K <= 512, d <= 128");
        return -1;
    }
#ifdef LSHKM_PHASE_TIMING
    static unsigned long long* prof_d = nullptr;
    if (!prof_d) (void)hipMalloc(&prof_d, 64);
    (void)hipMemsetAsync(prof_d, 0, 64, s);
    a.prof = prof_d;
    struct PhaseReport {      // printed after the launch sequence below
        hipStream_t s; unsigned long long* d;
        ~PhaseReport() {
            unsigned long long v[6];
            (void)hipMemcpyAsync(v, d, 48, hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
            // hi-only form: [0] load + split + hash, [1] centroid tiles, [2] certificate + chain + stores
            // (the LIST refinement's fused_persistent_kernel adds its own phases 0-4 over its few rows)
            fprintf(stderr, "PHASES %llu %llu %llu %llu %llu\n", v[0], v[1], v[2], v[3], v[4]);
        }
    } report{s, prof_d};
#endif
    const bool chunked = test_switch("LSHKM_FUSED_FORM", "chunked") && f.rows == 0;   // the streaming form (tests)
    const int npass = (f.Kpad + FP_KMAX - 1) / FP_KMAX;
    const bool multi_ok = npass == 1 || (f.part && f.part_bytes >= ((f.N + 31) / 32) * 64 * 16);
    // LIST refinement pass state: one slot per (segment, tile) of the list
    if (f.hi && npass > 1 && f.part_bytes < ((f.list_cap + 31) / 32 + FUSED_MAX_SEGS) * 64 * 16) {
        set_error("launch_fused: pass-state buffer too small for the refinement");
        return -1;
    }
    if (f.metric == 1 && (chunked || !multi_ok || !f.nbv || !f.hfix || !f.hfix_count || (hash && (!f.hi || f.k != 4)))) {
        set_error("launch_fused: cosine runs the persistent form only (hashing: the hi-only form with k = 4)");
        return -1;
    }
    if (f.metric == 1 && f.rows == 2 && !f.xn2) {
        set_error("launch_fused: cosine on fp64 rows needs the rows' sums of squares");
        return -1;
    }
    if (f.hi && (f.metric == 1 || !a.fast_dist) && (!f.cfix || !f.cfix_counts || !f.cfix_count)) {
        set_error("launch_fused: the hi-only cosine form needs the decline list, the exact euclidean one the pow fix-up list");
        return -1;
    }
    if (hash && (f.LK > 32 || f.L * f.k != f.LK)) {              // the fix-ups hold <= 32 functions per row
        set_error("launch_fused: hashing needs L * k <= 32");
        return -1;
    }
    if (!chunked && multi_ok && (!hash || f.k == 4)) {
        static int cus[64] = {0};
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return kstatus("hipGetDevice");
        if (dev < 64 && !cus[dev] &&
            hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return kstatus("hipDeviceGetAttribute");
        const int ncu = dev < 64 && cus[dev] > 0 ? cus[dev] : 256;
        const int64_t ntiles = (f.N + 31) / 32;
        const int64_t want = (ntiles + FP_WAVES - 1) / FP_WAVES;
        const int nblk = (int)std::max<int64_t>(1, std::min<int64_t>(ncu, want));
        const dim3 grid((unsigned)nblk), block(FP_THREADS);
        const int kslice = std::min(f.Kpad, FP_KMAX);
        const size_t lds = (size_t)fp_lds_bytes(kslice, hash);
        const size_t lds_nohash = (size_t)fp_lds_bytes(kslice, false);
        // list segments: block b's tiles hold at most FP_WAVES * 32 * ceil(tiles / (grid * FP_WAVES)) rows
        a.seg_rows = (int64_t)FP_WAVES * 32 * ((ntiles + (int64_t)nblk * FP_WAVES - 1) / ((int64_t)nblk * FP_WAVES));
        // the hi-only form strides by fh_waves() tiles per block (8 or 12)
        for (const int W : {FH_WAVES_MIN, FH_WAVES_MAX})
            a.seg_rows = std::max<int64_t>(a.seg_rows, (int64_t)W * 32 * ((ntiles + (int64_t)nblk * W - 1) / ((int64_t)nblk * W)));
        a.seg_counts = f.seg_counts;
        if (!f.seg_counts || f.seg_cap < nblk || (int64_t)nblk * a.seg_rows > f.list_cap) {
            set_error("launch_fused: list workspace too small");
            return -1;
        }
        f.nseg = nblk;
        f.seg_rows = a.seg_rows;
        if (hash && (!a.hfix || !a.hfix_count || (f.metric == 0 && !a.tuples) || f.LKpad > 32)) {   // pts[] holds 128 x 32 projections
            set_error("launch_fused: hashing needs the fix-up list, a tuple buffer and L*k <= 32");
            return -1;
        }
        if (f.metric == 1) { a.hfix = f.hfix; a.hfix_count = f.hfix_count; }
        a.part = reinterpret_cast<float4*>(f.part);
        a.list_in = nullptr; a.list_counts = nullptr; a.list_seg_rows = 0;
        f.final_list = f.ambig;
        f.final_counts = f.seg_counts;
        if (f.hi) {
            // hi-only passes (512 centroids each), the hash fix-up, then the
            // 3-product LIST form over the rows they listed (256 per pass)
            const bool cos = f.metric == 1;
            if (!f.list2 || !f.seg_counts2 || !f.refined || (f.Kpad > FH_KMAX && !f.part) || (cos && !f.hfix2)) {
                set_error("launch_fused: the hi-only form needs the second list and its counters");
                return -1;
            }
            const int np1 = (f.Kpad + FH_KMAX - 1) / FH_KMAX;
            a.ambig_count = f.refined;
            // 512 < K <= 1024, euclidean, LSHKM_HI_TWO_IMAGE=1: one two-image launch
            // instead of two passes with carried state. Measured at C5 (N = 10M,
            // K = 1024): 5.09 ms vs 1.83 + 2.51 ms, HBM 8.9 GB vs 13.8 GB per call --
            // the block-wide image swaps line the waves up and cost the MFMA/VALU
            // overlap between them, more than the second read of X costs; opt-in.
            const bool two_image = !cos && np1 == 2 && test_switch("LSHKM_HI_TWO_IMAGE", "1") && f.rows == 0;
            if (f.rows != 0) {
                // general rows: one hi-only pass (Kpad <= 512), then the LIST form below
                const size_t lh = (size_t)fh_lds_bytes(f.Kpad, false);
                const bool gath = f.rows == 1 && f.Kpad <= FH_GATH_KMAX && !test_switch("LSHKM_GATHER", "0");
#if defined(FH_WAVES_SET) && FH_WAVES_SET != 8
                if (gath) { set_error("launch_fused: gather ring needs 8 waves"); return -1; }
#else
                if (!cos && a.fast_dist)
                    hipLaunchKernelGGL((fused_hi_kernel<false, false, 0, 1, false, 1, true>), grid, dim3(64 * 8), lh, s, a);
                else if (gath && !cos)
                    hipLaunchKernelGGL((fused_hi_kernel<false, false, 0, 1, true, 1>), grid, dim3(64 * 8),
                                       (size_t)fh_gath_off(f.Kpad, false) + 8 * FH_GATH_WAVE, s, a);
                else
#endif
                if (cos && f.rows == 1)
                    hipLaunchKernelGGL((fused_hi_kernel<false, false, 1, 1, false, 1>), grid,
                                       dim3(64 * fh_waves<false, false, 1>()), lh, s, a);
                else if (cos)
                    hipLaunchKernelGGL((fused_hi_kernel<false, false, 1, 1, false, 2>), grid,
                                       dim3(64 * fh_waves<false, false, 1>()), lh, s, a);
                else if (f.rows == 1)
                    hipLaunchKernelGGL((fused_hi_kernel<false, false, 0, 1, false, 1>), grid,
                                       dim3(64 * fh_waves<false, false, 0>()), lh, s, a);
                else {
                    // the chain's pow buffers after the image when they fit (Kpad <= 448)
                    constexpr int PW_BYTES = fh_waves<false, false, 0>() * 512 * 8;
                    const size_t off = (lh + 255) & ~(size_t)255;
                    const bool pw = off + PW_BYTES <= 160 * 1024;
                    a.pw_lds = pw ? (int)off : 0;
                    hipLaunchKernelGGL((fused_hi_kernel<false, false, 0, 1, false, 2>), grid,
                                       dim3(64 * fh_waves<false, false, 0>()), pw ? off + PW_BYTES : lh, s, a);
                }
            }
            if (two_image) {
                a.Ch = f.Ch; a.cnh = f.cnh; a.Kpad = f.Kpad;
                a.t0 = 0; a.pass_first = 1; a.pass_last = 1;
                const size_t lh = (size_t)fh_lds_bytes(FH_KMAX, hash);
                if (hash) hipLaunchKernelGGL((fused_hi_kernel<true, false, 0, 2>), grid, dim3(64 * fh_waves<true, false, 0>()), lh, s, a);
                else hipLaunchKernelGGL((fused_hi_kernel<false, false, 0, 2>), grid, dim3(64 * fh_waves<false, false, 0>()), lh, s, a);
            }
            for (int p = 0; p < (two_image || f.rows != 0 ? 0 : np1); p++) {
                const int c0 = p * FH_KMAX;
                a.Ch = f.Ch + (size_t)c0 * FU_D; a.cnh = f.cnh + c0;
                a.Kpad = std::min(FH_KMAX, f.Kpad - c0);
                a.t0 = c0 / 32; a.pass_first = p == 0; a.pass_last = p == np1 - 1;
                const size_t lh = (size_t)fh_lds_bytes(a.Kpad, hash && p == 0);
#define FH_LAUNCH(H, M, C) \
    hipLaunchKernelGGL((fused_hi_kernel<H, M, C>), grid, dim3(64 * fh_waves<H, M, C>()), lh, s, a)
                if (cos) {
                    if (np1 == 1) {
                        if (hash) FH_LAUNCH(true, false, 1);
                        else FH_LAUNCH(false, false, 1);
                    } else {
                        if (hash && p == 0) FH_LAUNCH(true, true, 1);
                        else FH_LAUNCH(false, true, 1);
                    }
                } else if (np1 == 1) {
                    // K <= 256: the winner rows by the LDS-DMA gather (LSHKM_GATHER=0: register loads)
#if defined(FH_WAVES_SET) && FH_WAVES_SET != 8      // experiments: the gather ring is sized for 8 waves
                    if (false) {
#else
                    if (a.Kpad <= FH_GATH_KMAX && !test_switch("LSHKM_GATHER", "0")) {
                        const size_t lg = (size_t)fh_gath_off(a.Kpad, hash) + 8 * FH_GATH_WAVE;
                        // the certified f32 winner distance (a.fast_dist) compiled in
                        if (hash && a.fast_dist)
                            hipLaunchKernelGGL((fused_hi_kernel<true, false, 0, 1, false, 0, true>), grid,
                                               dim3(64 * fh_waves<true, false, 0, true>()), lh, s, a);
                        else if (a.fast_dist)
                            hipLaunchKernelGGL((fused_hi_kernel<false, false, 0, 1, false, 0, true>), grid,
                                               dim3(64 * fh_waves<false, false, 0, true>()), lh, s, a);
                        else if (hash)
                            hipLaunchKernelGGL((fused_hi_kernel<true, false, 0, 1, true>), grid, dim3(64 * 8), lg, s, a);
                        else hipLaunchKernelGGL((fused_hi_kernel<false, false, 0, 1, true>), grid, dim3(64 * 8), lg, s, a);
#endif
                    } else if (hash) {
                        FH_LAUNCH(true, false, 0);
                    } else {
                        FH_LAUNCH(false, false, 0);
                    }
                } else {
                    if (hash && p == 0) FH_LAUNCH(true, true, 0);
                    else if (a.fast_dist && a.pass_last)   // the winner's distance: certified f32, compiled in
                        hipLaunchKernelGGL((fused_hi_kernel<false, true, 0, 1, false, 0, true>), grid,
                                           dim3(64 * fh_waves<false, true, 0, true>()), lh, s, a);
                    else FH_LAUNCH(false, true, 0);
                }
#undef FH_LAUNCH
            }
            // the hash fix-up touches only tuples / phi / bucket of its listed rows:
            // on the side stream beside the LIST refinement when one is given
            const bool side = hash && f.side && f.fork && f.join;
            hipStream_t hs = side ? f.side : s;
            if (side) {
                if (hipEventRecord(f.fork, s) != hipSuccess || hipStreamWaitEvent(f.side, f.fork, 0) != hipSuccess)
                    return kstatus("launch_fused (fork)");
            }
            if (hash && cos) hipLaunchKernelGGL(hash_fixup_kernel<true>, dim3((unsigned)nblk * HF_SPLIT), dim3(64 * HF_WAVES), HF_LDS, hs, a);
            else if (hash) hipLaunchKernelGGL(hash_fixup_kernel<false>, dim3((unsigned)nblk * HF_SPLIT), dim3(64 * HF_WAVES), HF_LDS, hs, a);
            if (side && f.side_timing) {
                if (hipEventRecord(f.side_timing, f.side) != hipSuccess) {
                    (void)hipStreamSynchronize(f.side);
                    return kstatus("launch_fused (timing)");
                }
                f.side_timed = true;
            }
            if (side && hipEventRecord(f.join, f.side) != hipSuccess) {
                // never return with the fix-up unordered against later work on s
                (void)hipStreamSynchronize(f.side);
                return kstatus("launch_fused (join)");
            }
            FusedArgs r = a;
            r.list_in = f.ambig; r.list_counts = f.seg_counts; r.list_seg_rows = a.seg_rows;
            r.ambig = f.list2; r.seg_counts = f.seg_counts2; r.ambig_count = f.ambig_count;
            r.hfix = cos ? f.hfix2 : f.hfix; r.hfix_count = cos ? f.cfix_count : f.hfix_count;
            r.Cl = f.Cl;
            r.tuples = nullptr; r.phi = nullptr; r.bucket = nullptr;
            for (int p = 0; p < npass; p++) {
                const int c0 = p * FP_KMAX;
                r.Ch = f.Ch + (size_t)c0 * FU_D; r.Cl = f.Cl + (size_t)c0 * FU_D; r.cnh = f.cnh + c0;
                r.Kpad = std::min(FP_KMAX, f.Kpad - c0);
                r.t0 = c0 / 32; r.pass_first = p == 0; r.pass_last = p == npass - 1;
                if (cos && f.rows == 1) {
                    if (npass == 1) hipLaunchKernelGGL((fused_persistent_kernel<false, 1, false, true, 1>), grid, block, lds_nohash, s, r);
                    else hipLaunchKernelGGL((fused_persistent_kernel<false, 1, true, true, 1>), grid, block, lds_nohash, s, r);
                } else if (cos && f.rows == 2) {
                    if (npass == 1) hipLaunchKernelGGL((fused_persistent_kernel<false, 1, false, true, 2>), grid, block, lds_nohash, s, r);
                    else hipLaunchKernelGGL((fused_persistent_kernel<false, 1, true, true, 2>), grid, block, lds_nohash, s, r);
                } else if (cos) {
                    if (npass == 1) hipLaunchKernelGGL((fused_persistent_kernel<false, 1, false, true>), grid, block, lds_nohash, s, r);
                    else hipLaunchKernelGGL((fused_persistent_kernel<false, 1, true, true>), grid, block, lds_nohash, s, r);
                } else if (f.rows == 1) {
                    if (npass == 1) hipLaunchKernelGGL((fused_persistent_kernel<false, 0, false, true, 1>), grid, block, lds_nohash, s, r);
                    else hipLaunchKernelGGL((fused_persistent_kernel<false, 0, true, true, 1>), grid, block, lds_nohash, s, r);
                } else if (f.rows == 2) {
                    if (npass == 1) hipLaunchKernelGGL((fused_persistent_kernel<false, 0, false, true, 2>), grid, block, lds_nohash, s, r);
                    else hipLaunchKernelGGL((fused_persistent_kernel<false, 0, true, true, 2>), grid, block, lds_nohash, s, r);
                } else {
                    if (npass == 1) hipLaunchKernelGGL((fused_persistent_kernel<false, 0, false, true>), grid, block, lds_nohash, s, r);
                    else hipLaunchKernelGGL((fused_persistent_kernel<false, 0, true, true>), grid, block, lds_nohash, s, r);
                }
            }
            f.final_list = f.list2;
            f.final_counts = f.seg_counts2;
            if (!cos && !a.fast_dist && f.cfix) {      // the hi-only pass's pow fix-ups (exact distances)
                f.ncos_lists = 1;
                f.cos_list[0] = f.cfix; f.cos_counts[0] = f.cfix_counts;
            }
            if (cos) {
                f.ncos_lists = 2;
                f.cos_list[0] = f.cfix; f.cos_counts[0] = f.cfix_counts;
                f.cos_list[1] = f.hfix2; f.cos_counts[1] = f.seg_counts2;
            }
            if (side && f.defer_join) {
                f.join_pending = true;          // the caller joins (after its exact pass)
            } else if (side && hipStreamWaitEvent(s, f.join, 0) != hipSuccess) {
                (void)hipStreamSynchronize(f.side);
                return kstatus("launch_fused (join)");
            }
            return kstatus("fused_hi_kernel");
        }
        // one launch per 256-centroid slice (the hashing rides on the first)
        for (int p = 0; p < npass; p++) {
            const int c0 = p * FP_KMAX;
            a.Ch = f.Ch + (size_t)c0 * FU_D; a.Cl = f.Cl + (size_t)c0 * FU_D; a.cnh = f.cnh + c0;
            a.Kpad = std::min(FP_KMAX, f.Kpad - c0);
            a.t0 = c0 / 32; a.pass_first = p == 0; a.pass_last = p == npass - 1;
            if (npass == 1) {
                if (hash) hipLaunchKernelGGL((fused_persistent_kernel<true>), grid, block, lds, s, a);
                else if (f.metric == 1) hipLaunchKernelGGL((fused_persistent_kernel<false, 1>), grid, block, lds_nohash, s, a);
                else hipLaunchKernelGGL((fused_persistent_kernel<false>), grid, block, lds_nohash, s, a);
            } else {
                if (hash && p == 0) hipLaunchKernelGGL((fused_persistent_kernel<true, 0, true>), grid, block, lds, s, a);
                else if (f.metric == 1) hipLaunchKernelGGL((fused_persistent_kernel<false, 1, true>), grid, block, lds_nohash, s, a);
                else hipLaunchKernelGGL((fused_persistent_kernel<false, 0, true>), grid, block, lds_nohash, s, a);
            }
        }
        if (hash) hipLaunchKernelGGL(hash_fixup_kernel<false>, dim3((unsigned)nblk * HF_SPLIT), dim3(64 * HF_WAVES), HF_LDS, s, a);
        if (f.metric == 1) {
            f.ncos_lists = 1;
            f.cos_list[0] = f.hfix; f.cos_counts[0] = f.seg_counts;
        }
        return kstatus("fused_persistent_kernel");
    }
    const dim3 grid((unsigned)((f.N + FU_PB - 1) / FU_PB)), block(FU_THREADS);
    if (hash) hipLaunchKernelGGL(fused_kernel<true>, grid, block, FU_LDS_BYTES, s, a);
    else hipLaunchKernelGGL(fused_kernel<false>, grid, block, FU_LDS_BYTES, s, a);
    return kstatus("fused_kernel");
}

// Winners listed by the fused kernels for their distance alone: lane per row.
// Cosine (MET = 1): the certificate declined, the x87 chain decides
// (exact_cosine_x87_wave). Euclidean (MET = 0, exact distances): a square of
// the chain was inexact, so glibc's pow(x, 2) may differ from x*x -- the chain
// again with glibc's pow (exact_euclid_wave). CF_SPLIT blocks per list segment; both
// lists of a call (the hi-only pass's and the refinement's) in ONE launch, so
// the short list's lone chains (~40 us of latency) overlap the long one.
constexpr int CF_SPLIT = 8;
struct CosLists {
    const unsigned long long* list[2];
    const int32_t* counts[2];
};
template <typename TX, int MET>
__global__ __launch_bounds__(256) void cos_fix_seg_kernel(const TX* __restrict__ X, int d, const double* __restrict__ C,
                                                          CosLists cl, int nseg, int64_t seg_rows,
                                                          const int32_t* __restrict__ assign, double* __restrict__ dist,
                                                          const double* __restrict__ xn2, const double* __restrict__ nbv) {
    // consecutive blocks take different segments: blocks are dealt round-robin to
    // the 8 XCDs, and a short list fills only its segment's first part (with
    // seg = blockIdx / CF_SPLIT every busy block sat on one XCD: 4x slower)
    const int per_list = nseg * CF_SPLIT;
    const int li = blockIdx.x / per_list, b = blockIdx.x % per_list;
    const int seg = b % nseg, part = b / nseg;
    const int n = cl.counts[li][2 * seg + 1];
    const unsigned long long* l = cl.list[li] + (int64_t)seg * seg_rows;
    const bool vec = sizeof(TX) == 4 && d % 8 == 0 && ((uintptr_t)X & 15) == 0 && ((uintptr_t)C & 15) == 0;
    __shared__ double sqs[4][64 * 16];                   // gp_sq_wave: 64 * NV per wave
    double* sq = sqs[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    // wave-uniform trip count (the chains run the whole wave in step); a lane
    // past the list end repeats the wave's first row and writes nothing
    for (int i0 = part * 256 + (threadIdx.x & ~63); i0 < n; i0 += CF_SPLIT * 256) {
        const int i = i0 + lane;
        const bool live = i < n;
        const int64_t row = (int64_t)l[live ? i : i0];
        const TX* xr = X + row * d;
        const double* cr = C + (size_t)assign[row] * d;
        double v;
        if constexpr (MET == 1) {
            // the sums of squares precomputed (the prep's nbv; fp64 rows: row_sumsq)
            // when the launch has them: no squares left in the chain
            if (nbv && (sizeof(TX) == 4 || xn2)) {
                const double xa = sizeof(TX) == 4 ? -1.0 : xn2[row], cb = nbv[assign[row]];
                if (vec) v = exact_cosine_x87_pf<sizeof(TX) == 4>(xr, cr, d, xa, cb);
                else v = exact_cosine_x87_pf<false>(xr, cr, d, xa, cb);
            } else if (vec) {
                v = exact_cosine_x87_wave<sizeof(TX) == 4>(xr, cr, d, sq);
            } else {
                v = exact_cosine_x87_wave<false>(xr, cr, d, sq);
            }
        } else {
            if (vec) v = exact_euclid_wave<sizeof(TX) == 4>(xr, cr, d, sq);
            else v = exact_euclid_wave<false>(xr, cr, d, sq);
        }
        if (live) dist[row] = v;
    }
}

// out[i] = the reference's sum_j pow(x_ij, 2), j ascending (the |x|^2 of
// cosineDistance, cust_vector.hpp:148-151) for fp64 rows, lane per row. A wave
// takes 64 rows; VEC (d even, rows 16-B aligned): each 8-dim step of the 64
// rows is loaded as 16-B pieces, four lanes per row's 64 contiguous bytes, and
// transposed through LDS (a lane-per-row load touches 64 lines per instruction).
constexpr int RSQ_S = 10;                                // LDS row stride (doubles)
template <bool VEC>
__global__ __launch_bounds__(256) void row_sumsq_kernel(const double* __restrict__ X, int64_t N, int d,
                                                         double* __restrict__ out) {
    __shared__ double sqs[4][64 * 8];                    // gp_sq_wave: 64 * NV per wave
    __shared__ __attribute__((aligned(16))) double tr[4][64 * RSQ_S];
    double* sq = sqs[threadIdx.x >> 6];
    double* t = tr[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    // wave-uniform trip count: lanes past N repeat row N - 1 and write nothing
    for (int64_t i0 = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63); i0 < N; i0 += (int64_t)gridDim.x * 256) {
        const int64_t i = i0 + lane;
        double a = 0.0;
        if constexpr (VEC) {
            double2 pc[4], pn[4];
            auto load = [&](int j0, double2 (&dst)[4]) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int q = 64 * k + lane, r = q >> 2, part = q & 3;
                    const int64_t rr = i0 + r < N ? i0 + r : N - 1;
                    const int j = j0 + 2 * part;
                    dst[k] = j < d ? *reinterpret_cast<const double2*>(X + rr * d + j) : make_double2(0.0, 0.0);
                }
            };
            load(0, pn);
            for (int j0 = 0; j0 < d; j0 += 8) {
#pragma unroll
                for (int k = 0; k < 4; k++) pc[k] = pn[k];
                if (j0 + 8 < d) load(j0 + 8, pn);               // the next step in flight
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int q = 64 * k + lane;
                    *reinterpret_cast<double2*>(t + (q >> 2) * RSQ_S + 2 * (q & 3)) = pc[k];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                double v[8], p[8];
#pragma unroll
                for (int h = 0; h < 4; h++) {
                    const double2 w = *reinterpret_cast<const double2*>(t + lane * RSQ_S + 2 * h);
                    v[2 * h] = w.x;
                    v[2 * h + 1] = w.y;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                gp_sq_wave<8>(v, p, sq);
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (j0 + u < d) a = __dadd_rn(a, p[u]);
            }
        } else {
            const double* x = X + (i < N ? i : N - 1) * d;
            for (int j0 = 0; j0 < d; j0 += 8) {
                double v[8], p[8];
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = j0 + u < d ? x[j0 + u] : 0.0;
                gp_sq_wave<8>(v, p, sq);
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (j0 + u < d) a = __dadd_rn(a, p[u]);
            }
        }
        if (i < N) out[i] = a;
    }
}

int launch_row_sumsq(hipStream_t s, const double* X, int64_t N, int d, double* out) {
    if (N <= 0) return 0;
    const unsigned grid = (unsigned)std::min<int64_t>((N + 255) / 256, 4096);
    if (d % 2 == 0 && ((uintptr_t)X & 15) == 0) hipLaunchKernelGGL(row_sumsq_kernel<true>, dim3(grid), dim3(256), 0, s, X, N, d, out);
    else hipLaunchKernelGGL(row_sumsq_kernel<false>, dim3(grid), dim3(256), 0, s, X, N, d, out);
    return kstatus("row_sumsq_kernel");
}

int launch_cos_fix_seg(hipStream_t s, Pts X, int d, const double* C, int nlists, const unsigned long long* const* lists,
                       const int32_t* const* counts, int64_t seg_rows, int nseg, const int32_t* assign, double* dist,
                       int metric, const double* xn2, const double* nbv) {
    if (nseg <= 0 || nlists <= 0) return 0;
    if (nlists > 2) return -1;                       // LSHKM_ERR_ARG
    CosLists cl{};
    for (int i = 0; i < nlists; i++) { cl.list[i] = lists[i]; cl.counts[i] = counts[i]; }
    const dim3 grid((unsigned)(nlists * nseg * CF_SPLIT));
#define CF_LAUNCH(TX, M, XP) hipLaunchKernelGGL((cos_fix_seg_kernel<TX, M>), grid, dim3(256), 0, s, XP, d, C, cl, nseg, seg_rows, assign, dist, xn2, nbv)
    if (metric == 1) {
        if (X.f64) CF_LAUNCH(double, 1, X.d()); else CF_LAUNCH(float, 1, X.f());
    } else {
        if (X.f64) CF_LAUNCH(double, 0, X.d()); else CF_LAUNCH(float, 0, X.f());
    }
#undef CF_LAUNCH
    return kstatus("cos_fix_seg_kernel");
}

}  // namespace lshkm
