// fused_args.h — the argument block of the fused hash + assign kernels
// (fused.hip: the persistent and hi-only forms).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tile.h"

namespace lshkm {

struct FusedArgs {
    const float* X;
    int64_t N;
    // centroids (prepared by fused_centroid_prep)
    const _Float16* Ch;
    const _Float16* Cl;
    const float* cnh;        // [Kpad] -||c||^2 / 2 (f32), -inf for padding rows
    const float* cbound;     // [0] = ec (times |x|), [1] = eb (constant), [2] = range flag (bits), [3] = max |c|,
                             // [4] = max |c - ch|, [5] = max |ch|, [6] = max |c|^2 / 2 (all rounded up),
                             // [7] = nonzero if some centroid value is not an f32 (bits)
    const double* C64;       // [K][128] exact centroids
    int Kpad;
    // hash family (HASH only)
    const _Float16* Vh;      // [32][128] f16 hi of the projections (rows >= LK zero)
    const _Float16* Vl;
    const double* PT;        // [128][LKpad] fp64 projections (exact paths)
    const float* tv;         // [LK]
    const double* pnorm;     // [LK] ||v||_2 (rounded up)
    const double* v1;        // [LK] ||v||_1 (rounded up)
    const int32_t* rv;       // [LK]
    float w;
    int L, k, LK, LKpad;
    int64_t nb;
    // outputs
    int32_t* tuples;         // [N][L][k] (may be null)
    int32_t* phi;            // [N][L] (may be null)
    int32_t* bucket;         // [N][L] (may be null)
    int32_t* assign;         // [N]
    double* dist;            // [N]
    int32_t* ambig;          // [N] uncertified rows
    unsigned long long* ambig_count;
    unsigned long long* hfix;        // persistent form: rows with an uncertified floor
    unsigned long long* hfix_count;
    // hi-only cosine form: rows whose winner distance the certified quotient
    // declined (cos_fix_seg pass); counts in cfix_counts[2b + 1]
    unsigned long long* cfix;
    int32_t* cfix_counts;
    unsigned long long* cfix_count;
    unsigned long long* stats;
    // persistent form: block b owns ambig/hfix entries [b * seg_rows, (b+1) * seg_rows)
    // and reports their counts in seg_counts[2b] (ambiguous), seg_counts[2b+1] (fix-up)
    int64_t seg_rows;
    int32_t* seg_counts;
    BucketDiv bdiv;          // phi % nb by multiply-high
    const double* nbv;       // cosine: [K] sequential sum of c_j^2 (cust_vector.hpp:139-155)
    const double* xn2;       // cosine, fp64 rows: [N] the rows' sequential sum of pow(x_j, 2)
    // multi-pass persistent form (K > 256): this launch scores centroid tiles
    // t0.. of the slice in Ch/Cl/cnh (Kpad rows); the running state per lane
    // crosses passes in part[tile * 64 + lane]
    float4* part;
    int t0, pass_first, pass_last;
    // LIST form (refinement of the rows a hi-only pass left uncertified): block b
    // takes the rows list_in[b * list_seg_rows ..][0 .. list_counts[2b])
    const int32_t* list_in;
    const int32_t* list_counts;
    int64_t list_seg_rows;
    unsigned long long* prof;        // LSHKM_PHASE_TIMING builds only: per-phase wave cycles
    const float* C32;                // fast_dist: [Kpad][128] f32(c) and |c - f32(c)| (FusedLaunch)
    const float* rn32;
    int fast_dist;
    // general rows (fused_hi_kernel<..., ROWS = 1 / 2>): fp32 (X) or fp64 (X64)
    // rows of d <= 128 dims, row stride d; xvec: rows 16-B aligned (vector loads)
    const double* X64;
    int d, xvec;
    const double* Cd;                // general rows: the caller's [K][d] centroids (cosine winners)
    int pw_lds;                      // fp64 rows, exact distances: LDS byte offset of the chain's
                                     // gp_sq_wave buffers (4 KiB per wave), 0: PwAcc + fix-up list
};

}  // namespace lshkm
