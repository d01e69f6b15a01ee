// kernels.h — launchers of the gfx950 kernels (host-callable, stream-ordered).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lshkm {

// Projection families, one launcher (hash.hip).
enum HashMode {
    HM_LSH_EUCLID = 0,    // EuclideanPhiGen: tuples + phi + bucket
    HM_LSH_COSINE = 1,    // CosineGGen: g (= phi = bucket)
    HM_CUBE_EUCLID_H = 2, // EuclideanFGen's inner h values [N][k]
    HM_CUBE_COSINE = 3,   // HypercubeGen over CosineHGen: vertex [N]
};

struct HashParams {
    const double* PT;     // [d][LKpad] projections, transposed (fp32 V widened exactly, or fp64 R)
    const float* t;       // [LK]   (euclidean)
    const double* pnorm;  // [LK]   ||projection||_2, rounded up
    const int32_t* r;     // [LK]   (LSH euclidean)
    float w;
    int d, L, k, LK, LKpad;
    int dstride;          // LDS row stride (floats): d rounded up to 4, plus 4
    int64_t nb;
};
int hash_fb(int LK);      // projections per accumulator block
int hash_lkpad(int LK);   // padded PT row length

int launch_proj_hash(hipStream_t s, int mode, const float* X, int64_t N, const HashParams& p,
                     int32_t* out_h, int32_t* out_phi, int32_t* out_bucket,
                     unsigned long long* stats);

// Lloyd assignment (assign.hip).
struct AssignWorkspace {
    float* C32;          // [Kpad][DP]
    float* cconst;       // [3][Kpad]  cn2, ecoef, eb
    int32_t* ambig;      // [N] list of uncertified rows
    unsigned long long* counters;  // [0] = ambiguous count (device)
};
int assign_dp(int d);    // padded dimension used by the MFMA kernel (0 = unsupported)
int launch_centroid_prep(hipStream_t s, const double* C, int K, int Kpad, int d, int DP, int metric,
                         float* C32, float* cconst);
int launch_assign_mfma(hipStream_t s, const float* X, int64_t N, int d, int DP, const double* C, int K,
                       int Kpad, const float* C32, const float* cconst, int32_t* assign, double* dist,
                       int32_t* ambig, unsigned long long* ambig_count);
int launch_assign_exact(hipStream_t s, const float* X, int64_t N, int d, const double* C, int K,
                        int metric, const int32_t* rows, const unsigned long long* row_count,
                        int64_t max_rows, int32_t* assign, double* dist);
int launch_assign_override(hipStream_t s, const int32_t* src_rows, int K, int64_t N, int32_t* assign,
                           double* dist);

int launch_add_counter(hipStream_t s, unsigned long long* dst, const unsigned long long* src);

// Synthetic data.
int launch_synth(hipStream_t s, uint64_t seed, int64_t row0, int64_t rows, int d, float* X);

}  // namespace lshkm
