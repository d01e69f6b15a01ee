// kernels.h — launchers of the gfx950 kernels (host-callable, stream-ordered).
#pragma once
#include <climits>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lshkm {

// Dataset rows in HBM: fp32 (the storage the hot path is tuned for: the
// synthetic / proj-2 values are fp32-representable) or fp64 (general doubles,
// e.g. the recommender's user vectors, crypto_rec.hpp:78-140).
// Kernels that read rows are templated on the element type; launchers take a
// Pts and dispatch.
struct Pts {
    const void* p = nullptr;
    bool f64 = false;
    Pts() = default;
    Pts(const float* x) : p(x), f64(false) {}
    Pts(const double* x) : p(x), f64(true) {}
    const float* f() const { return static_cast<const float*>(p); }
    const double* d() const { return static_cast<const double*>(p); }
    size_t esize() const { return f64 ? 8 : 4; }
    // row r of a [.][d] matrix
    Pts row(int64_t r, int d) const {
        Pts q = *this;
        q.p = static_cast<const char*>(p) + (size_t)r * d * esize();
        return q;
    }
};

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
    int64_t nb;
};
int hash_fb(int LK);      // projections per accumulator block
int hash_lkpad(int LK);   // padded PT row length

int launch_proj_hash(hipStream_t s, int mode, Pts X, int64_t N, const HashParams& p,
                     int32_t* out_h, int32_t* out_phi, int32_t* out_bucket,
                     unsigned long long* stats);

// Split-f16 MFMA hashing (hash_mfma.hip): fp32 points, d = 128, L*k <= 32.
struct HashMfmaParams {
    const _Float16* Vh;   // [>= 32][128] f16 hi of the projections (rows >= LK zero)
    const _Float16* Vl;   // lo
    const float* t;       // [LK] (euclidean)
    const double* pnorm;  // [LK] |v|_2 rounded up
    const double* v1;     // [LK] |v|_1 rounded up
    const int32_t* r;     // [LK] (LSH euclidean)
    const double* PT;     // [d][LKpad] fp64 projections (the fix-up pass)
    float w;
    int d, L, k, LK, LKpad;
    int64_t nb;
};
// out_h: LSH euclidean tuples [N][L*k] / cube euclidean h [N][k] / cube cosine
// vertex [N]; mm: cube euclidean h range (atomicMin/Max into a pre-set pair).
// list / seg_counts: per-block lists of the uncertified rows (workspace).
int launch_hash_mfma(hipStream_t s, int mode, const float* X, int64_t N, const HashMfmaParams& p, int32_t* out_h,
                     int32_t* out_phi, int32_t* out_bucket, int32_t* mm, unsigned long long* list, int64_t list_cap,
                     int32_t* seg_counts, int seg_cap, unsigned long long* stats, int h16 = 0);

// Lloyd assignment (assign.hip).
struct AssignWorkspace {
    float* C32;          // [Kpad][DP]
    float* cconst;       // [3][Kpad]  cn2, ecoef, eb
    int32_t* ambig;      // [N] list of uncertified rows
    unsigned long long* counters;  // [0] = ambiguous count (device)
};
int assign_dp(int d);    // padded dimension used by the MFMA kernel (0 = unsupported)
int launch_centroid_prep(hipStream_t s, const double* C, int K, int Kpad, int d, int DP, int metric, bool xf64,
                         float* C32, float* cconst);
int launch_assign_mfma(hipStream_t s, Pts X, int64_t N, int d, int DP, const double* C, int K,
                       int Kpad, int metric, const float* C32, const float* cconst, int32_t* assign, double* dist,
                       int32_t* ambig, unsigned long long* ambig_count);
// Lloyd cosine winners whose distance the certified form declined (list at
// rows[0..*count), written by assign_mfma_kernel<., 1>): soft-x87 distances.
int launch_cos_fix(hipStream_t s, Pts X, int64_t N, int d, const double* C, const int32_t* rows,
                   const unsigned long long* count, const int32_t* assign, double* dist);
int launch_assign_exact(hipStream_t s, Pts X, int64_t N, int d, const double* C, int K,
                        int metric, const int32_t* rows, const unsigned long long* row_count,
                        int64_t max_rows, int32_t* assign, double* dist, const int32_t* seg_counts = nullptr,
                        int64_t seg_rows = 0, int nseg = 0, const double* xn2 = nullptr, const double* nbv = nullptr);
// Euclidean, listed rows, batched (CT: d * ceil64(K) doubles of workspace).
// Segmented form (seg_counts != NULL): segment b = rows[b * seg_rows ...], count seg_counts[2b].
int launch_assign_exact_list(hipStream_t s, Pts X, int d, const double* C, int K, double* CT,
                             const int32_t* rows, const unsigned long long* row_count, int64_t max_rows,
                             int32_t* assign, double* dist, const int32_t* seg_counts = nullptr,
                             int64_t seg_rows = 0, int nseg = 0);
// Euclidean, listed rows, K <= 1024: f32 candidate pruning, then exact order on
// the candidates only (ws: d * ceil64(K) + ceil64(K) + ceil64(K)/32 floats).
// exact_dist = 0 (LSHKM_DIST_CERTIFIED): a winner distance may come from the
// x*x chain (<= 2^-44 relative); cluster IDs are the reference's either way.
int launch_assign_pruned_list(hipStream_t s, Pts X, int d, const double* C, int K, float* ws,
                              const int32_t* rows, const unsigned long long* row_count, int64_t max_rows,
                              int32_t* assign, double* dist, const int32_t* seg_counts = nullptr,
                              int64_t seg_rows = 0, int nseg = 0, int metric = 0, int exact_dist = 1,
                              bool prepped = false);
// The centroid-only part of the pruned pass (f32 transposed centroids, |c|^2,
// the chunk bounds into ws): launched before the fused pass, off its tail;
// then launch_assign_pruned_list(..., prepped = true).
int launch_assign_pruned_prep(hipStream_t s, bool xf64, int d, const double* C, int K, float* ws, int metric);
int launch_assign_override(hipStream_t s, const int32_t* src_rows, int K, int64_t N, int32_t* assign,
                           double* dist);

int launch_add_counter(hipStream_t s, unsigned long long* dst, const unsigned long long* src);
// stats[dst_idx[i]] += *src[i], i < n <= 8, in one launch
int launch_add_counters(hipStream_t s, unsigned long long* stats, int n, const int* dst_idx,
                        const unsigned long long* const* src);

// Stable bucket scatter (scatter.hip).
size_t sort_scratch_bytes(int64_t N, int64_t range, int T = 1);
// Distinct int32 keys, n <= 8192: one-workgroup bitonic sort of (key, val) pairs.
// n_dev: the count is read on the device instead; n is then the caller's bound on
// it (refused past 8192).
// The pow contract (pow2.hip): lshkm_pow_selfcheck once per process; 0, or
// LSHKM_ERR_UNSUPPORTED with the error set when this process's pow differs.
int pow_contract_check();

int sort_pairs_small(hipStream_t s, const int32_t* keys, const int32_t* vals, int64_t n, int32_t* keys_out,
                     int32_t* vals_out, const unsigned int* n_dev = nullptr);
int stable_sort_by_key(hipStream_t s, const int32_t* keys, int64_t kstride, const int32_t* vals, int64_t N,
                       int64_t range, int32_t* keys_out, int32_t* vals_out, void* scratch);
int launch_csr_bounds(hipStream_t s, const int32_t* sorted_keys, int64_t N, int64_t nb, int64_t* row_ptr, int T = 1);
// T independent stable sorts in one set of launches (table t: keys + t * key_ts,
// vals + t * val_ts; outputs at + t * N).
int stable_sort_by_key_batched(hipStream_t s, const int32_t* keys, int64_t kstride, int64_t key_ts, const int32_t* vals,
                               int64_t val_ts, int T, int64_t N, int64_t range, int32_t* keys_out, int32_t* vals_out,
                               void* scratch);

// Queries (query.hip).
size_t scan_ws_bytes(int64_t M);
int launch_scan_i64(hipStream_t s, const int64_t* a, int64_t M, int64_t* out, int64_t* scratch = nullptr);
int launch_lsh_query(hipStream_t s, const int32_t* qbucket, const int32_t* qtuple, const int32_t* alias, int64_t nq,
                     int L, int k, int64_t nb, int filtered, int64_t N, const int32_t* tuples, const int32_t* bucket,
                     const int64_t* row_ptr, const int32_t* idx, int64_t* sizes, int64_t* cand_off,
                     int32_t* klist, int64_t* kcount, int64_t* qsz, int64_t* out_ptr, int32_t* out, int phase,
                     int64_t* scan_ws = nullptr, const int32_t* mt0 = nullptr);
int launch_lsh_gather_t0(hipStream_t s, const int32_t* tuples, const int32_t* idx, int64_t N, int L, int k, int32_t* mt0);
int launch_cube_query(hipStream_t s, const int32_t* qvert, int64_t nq, const int32_t* masks, int S,
                      const int64_t* row_ptr, const int32_t* idx, int64_t* sizes, int64_t* slot_off,
                      int64_t* out_ptr, int32_t* out, int64_t* scan_ws = nullptr);

// Hypercube coins (cube.hip).
int launch_h_minmax(hipStream_t s, const int32_t* h, int64_t n, int32_t* mm_dev);
// h: int32 [N][k], or int16 when h16 (the hash kernel's narrow output).
int launch_coin_first(hipStream_t s, const void* h, bool h16, int64_t N, int k, int32_t hmin, int32_t hspan,
                      const int32_t* memo, int32_t* first_row);
int launch_coin_collect(hipStream_t s, int32_t* first_row, int64_t total, int k, int32_t hspan, int32_t* keys,
                        int32_t* vals, unsigned int* count);
int launch_coin_draw(hipStream_t s, const int32_t* sorted_vals, const unsigned int* count, int32_t hmin, int32_t hspan,
                     int32_t* memo, uint32_t* state);
int launch_coin_vertex(hipStream_t s, const void* h, bool h16, int64_t N, int k, int32_t hmin, int32_t hspan,
                       const int32_t* memo, int32_t* vertex);
int launch_memo_rehome(hipStream_t s, const int32_t* old_memo, int32_t old_min, int32_t old_span, int32_t* new_memo,
                       int32_t new_min, int32_t new_span, int k);
int launch_memo_scatter(hipStream_t s, const int32_t* off, const int32_t* bit, int64_t n, int32_t* memo);

// k-means update (update.hip).
// carry / carry_counts (may be NULL): the running sums and counts the chain
// continues from (exact-order sharded mode).
int launch_km_chain(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K,
                    double* sums, int64_t* counts, const double* carry = nullptr,
                    const int64_t* carry_counts = nullptr);
// The same sums by binade segments (kmseg.h; ws: km_seg_ws_bytes): every chain
// of fp64 rows; flag != NULL: only the flagged (cluster, 64-dim block) chains.
size_t km_seg_ws_bytes(int64_t M, int K, int d);
// above this the update takes the fixed-point form instead (same exact sums)
constexpr size_t KM_SEG_WS_CAP = (size_t)8 << 30;
int launch_km_sums_seg(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                       double* sums, int64_t* counts, const double* carry, const int64_t* carry_counts, void* ws,
                       const int* flag = nullptr);
// Same sums, parallel: plain fp64 adds in any order wherever the sequential
// chain provably never rounds (km_cert), the rounding chains by segments
// (seg_ws: km_seg_ws_bytes) or, without seg_ws, by the sequential kernel
// (ws: km_fx_ws_bytes). stat: counts the chains the test flags.
size_t km_fx_ws_bytes(int K, int d);
int launch_km_sums_fx(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                      double* sums, int64_t* counts, const double* carry, const int64_t* carry_counts, void* ws,
                      unsigned long long* stat = nullptr, void* seg_ws = nullptr);
// Sharded form (lshkm_kmeans_shard_*): begin (ws: km_shard_ws_bytes), certify,
// prepare / chain (the flagged chains' records and their composition).
size_t km_shard_ws_bytes(int64_t M, int K, int d);
int launch_km_shard_begin(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                          double* sums, double* asum, int32_t* qt, int64_t* counts, void* ws);
int launch_km_shard_certify(hipStream_t s, const double* gathered, int world, int rank, const double* asum,
                            const int32_t* qt, const int64_t* counts, int K, int d, double* sums_out, double* start,
                            int* flag, uint8_t* mask, unsigned long long* nflag);
int launch_km_shard_prepare(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                            const double* start, const int* flag, const uint8_t* mask, void* ws);
int launch_km_shard_chain(hipStream_t s, Pts X, int d, const int32_t* rows, const int64_t* crow, int K, int64_t M,
                          const int* flag, const uint8_t* mask, const double* carry, void* ws, double* sums);
// Column chains of K row blocks [crow[k], crow[k+1]) of a row-major [n][m]
// fp64 matrix (row order, from carry [K][m] or 0; iota from launch_seg_iota;
// ws: seg_columns_ws_bytes) by binade segments -> out [K][m].
size_t seg_columns_ws_bytes(int64_t n, int K, int m);
int launch_seg_iota(hipStream_t s, int32_t* iota, int64_t n);
int launch_seg_columns(hipStream_t s, const double* V, int64_t n, int K, int m, const int32_t* iota,
                       const int64_t* crow, const double* carry, double* out, void* ws);
// Grid test of a matrix's values (update.hip): qt [3] device ints; after the
// copy back, grid_exact_squares says whether every difference of two values
// squares exactly with pow(x, 2) == x*x.
int launch_grid_bits(hipStream_t s, Pts X, int64_t n, int* qt);
bool grid_exact_squares(const int* qt_host);
int launch_km_finalize(hipStream_t s, const double* sums, const int64_t* counts, int K, int d, const double* C_old,
                       int metric, double min_dist, double* C_new, int* moved);

// k-means++ seeding (kmeanspp.hip): iterations 1..K-1 on the stream.
// chosen[0] and canon[1..K-1] (the engine's canonical draws) already on the
// device; ws holds kmeans_pp_ws_bytes(N) bytes.
size_t kmeans_pp_ws_bytes(int64_t N);
int launch_kmeans_pp(hipStream_t s, Pts X, int64_t N, int d, int K, int metric, const double* canon,
                     int32_t* chosen, void* ws, unsigned long long* stats);

// Recommend step (recom.hip): fp64 rows, per-user candidate CSR.
int launch_rc_norms(hipStream_t s, const double* X, int64_t N, int d, double* xa);
int launch_rc_cluster_top_n(hipStream_t s, Pts X, const double* x_mean, int d, const int64_t* crow,
                            const int32_t* crows, int K, Pts U, const double* u_mean, int64_t nq, const int32_t* ucl,
                            const int64_t* unk_ptr, const int32_t* unk_idx, int n_top, double* scratch,
                            int64_t scratch_row, int nwaves, double* pred, int32_t* pidx, int32_t* out,
                            unsigned long long* soft_count);
// The terms form of the clustering recommender (recom.hip): similarities and
// the per-(member, unknown index) terms of every user at once, then the chains
// one wave per user (its chains lane by lane), then the quicksort per user.
int rc_terms_stride8(int d, int elem);
// Cluster-major work list of the terms form (rc_terms_cl_kernel): group g =
// the users gusr[gptr[g] .. gptr[g + 1]) of cluster gcl[g]; its 64-member
// chunks are the items ioff[g] .. ioff[g + 1] - 1 (nitems = ioff[ngroups]).
struct RcGroups {
    const int32_t* ioff;
    int ngroups;
    int64_t nitems;
    const int32_t* gcl;
    const int32_t* gptr;
    const int32_t* gusr;
    void* items;              // nitems x 32 B (16-B aligned): the per-item records (rc_item_meta_kernel)
    int64_t nusers;           // gptr[ngroups]: the work list's users
    void* users;              // nusers x 48 B (16-B aligned): the per-user records (rc_user_meta_kernel)
};
constexpr size_t RC_ITEM_BYTES = 32, RC_USER_BYTES = 48;
int launch_rc_terms(hipStream_t s, Pts X, const double* x_mean, int d, const int64_t* crow, const int32_t* crows,
                    int K, Pts U, int64_t nq, const int32_t* ucl, const int64_t* soff, int64_t total,
                    const int64_t* unk_ptr, const int32_t* unk_idx, const int64_t* toff, double* sims, double* terms,
                    int32_t* mem_q, int32_t* mem_r, int64_t* fix_list, unsigned long long* fix_count,
                    unsigned long long* soft_count, double* unorm, const RcGroups* groups, int64_t* fix_region,
                    int64_t* fix_aux);
// fix_region: total entries (the terms blocks' private decline lists); fix_aux: 2 x RC_TERMS_GMAX
constexpr int RC_TERMS_GMAX = 8192;
// Users whose cluster holds >= RC_LONG_MIN members on this shard: their
// prediction chains by binade segments (launch_seg_columns, all such users in
// one set of launches) instead of one wave's sequential adds. Device
// workspace: tab [nlong] RcLongUser, crow [nlong + 1] (row offsets in V), V
// [rows][D] (D = max m + 1: each user's terms, zero-padded, then |sim|),
// iota [rows], carry / sums [nlong][D], ws (seg_columns_ws_bytes).
constexpr int64_t RC_LONG_MIN = 16384;
struct RcLongUser {
    int64_t q, n, b0, toff, u0, m, off, pad;
};
struct RcLong {
    const RcLongUser* tab;
    int64_t nlong, rows;
    int D;
    const int64_t* crow;
    double *V, *carry, *sums;
    int32_t* iota;
    void* ws;
};
int launch_rc_chain_terms(hipStream_t s, int64_t nq, const int64_t* soff, const int64_t* unk_ptr, const int64_t* toff,
                          const double* sims, const double* terms, const double* carry_main, const double* carry_abs,
                          const int64_t* carry_cnt, const double* u_mean, double* main_out, double* abs_out,
                          int64_t* cnt_out, double* pred, int64_t long_min = INT64_MAX);
int launch_rc_long(hipStream_t s, const double* sims, const double* terms, const double* carry_main,
                   const double* carry_abs, const int64_t* carry_cnt, const double* u_mean, double* main_out,
                   double* abs_out, int64_t* cnt_out, double* pred, const RcLong& lng);
int launch_rc_top(hipStream_t s, int64_t nq, const int64_t* soff, const int64_t* carry_cnt, const int64_t* unk_ptr,
                  const int32_t* unk_idx, double* pred, int32_t* pidx, int n_top, int32_t* out);
constexpr int RC_CLUSTER_WAVES_PER_BLOCK = 4;     // rc_cluster_top_n_kernel: waves per block (RC_WAVES)
int launch_rc_shard_sims(hipStream_t s, Pts X, int d, const int64_t* crow, const int32_t* crows, int K, Pts U,
                         int64_t nq, const int32_t* ucl, const int64_t* unk_ptr, const int64_t* soff, double* sims,
                         unsigned long long* soft_count);
int launch_rc_shard_chain(hipStream_t s, Pts X, const double* x_mean, int d, const int64_t* crow, const int32_t* crows,
                          int K, int64_t nq, const int32_t* ucl, const double* u_mean, const int64_t* unk_ptr,
                          const int32_t* unk_idx, const int64_t* soff, const double* sims, const double* carry_main,
                          const double* carry_abs, const int64_t* carry_cnt, double* main_out, double* abs_out,
                          int64_t* cnt_out, int n_top, double* pred, int32_t* pidx, int32_t* out);
int launch_rc_p_closest(hipStream_t s, const double* X, const double* xa, int d, const double* U, int64_t nq,
                        const int64_t* cand_ptr, const int32_t* cand_idx, int P, double* sim, double* key,
                        int32_t* pos, int32_t* out_idx, double* out_sim, int32_t* out_cnt, int32_t* replay,
                        unsigned int* replay_count);
int launch_rc_top_n(hipStream_t s, const double* X, const double* x_mean, int d, const double* u_mean, int64_t nq,
                    const int64_t* unk_ptr, const int32_t* unk_idx, const int32_t* nb_idx, const double* nb_sim,
                    const int32_t* nb_cnt, int P, int n_top, double* pred, int32_t* pidx, int32_t* out);

// Fused hash + assign on split-f16 MFMA (fused.hip), d = 128.
struct FusedLaunch {
    // optional side stream (+ fork / join events): the hash fix-up runs there
    // beside the LIST refinement; joined before launch_fused returns, or, with
    // defer_join, left to the caller (out: join_pending = the main stream must
    // still wait on `join` -- the caller's exact pass then also overlaps it)
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    bool defer_join = false;
    bool join_pending = false;
    hipEvent_t side_timing = nullptr;            // recorded on the side stream after the fix-up (timing)
    bool side_timed = false;                     // out: side_timing was recorded by this launch
    const float* X = nullptr;
    int64_t N = 0;
    const _Float16* Ch = nullptr;
    const _Float16* Cl = nullptr;
    const float* cnh = nullptr;
    const float* cbound = nullptr;
    const double* C64 = nullptr;
    int Kpad = 0;
    const _Float16* Vh = nullptr;
    const _Float16* Vl = nullptr;
    const double* PT = nullptr;
    const float* tv = nullptr;
    const double* pnorm = nullptr;
    const double* v1 = nullptr;
    const int32_t* rv = nullptr;
    float w = 0.f;
    int L = 0, k = 0, LK = 0, LKpad = 0;
    int64_t nb = 1;
    int32_t* tuples = nullptr;
    int32_t* phi = nullptr;
    int32_t* bucket = nullptr;
    int32_t* assign = nullptr;
    double* dist = nullptr;
    int32_t* ambig = nullptr;
    unsigned long long* ambig_count = nullptr;
    unsigned long long* hfix = nullptr;          // (row << 32 | fn mask) of uncertified hashes
    unsigned long long* hfix_count = nullptr;
    unsigned long long* stats = nullptr;
    // persistent form: ambig / hfix are split in per-block segments
    int64_t list_cap = 0;                        // entries available in ambig and in hfix
    int32_t* seg_counts = nullptr;               // [2 * seg_cap]
    int seg_cap = 0;
    // out: nseg > 0 when the lists are segmented (segment b = [b * seg_rows, ...))
    int nseg = 0;
    int64_t seg_rows = 0;
    // cosine Lloyd (metric 1, no hashing): nbv[c] = the reference's sequential
    // sum of c_j^2; hfix/hfix_count then list the rows whose winner distance the
    // certified form declined (cos_fix_seg pass)
    int metric = 0;
    const double* nbv = nullptr;
    const double* xn2 = nullptr;    // cosine, fp64 rows: [N] sum_j pow(x_j, 2) (launch_row_sumsq)
    // euclidean fast distance (fast_dist): the winner's distance from f32(c) in
    // f32, certified to 2^-20 relative (else the row is refined exactly);
    // C32 [Kpad][128] = f32(c), rn32 [Kpad] = |c - f32(c)|_2 rounded up
    const float* C32 = nullptr;
    const float* rn32 = nullptr;
    int fast_dist = 0;
    // general rows (euclidean Lloyd, no hashing, Kpad <= 512): rows = 1: fp32
    // rows of d <= 128 dims (X); rows = 2: fp64 rows of d <= 128 dims (X64).
    // C64 is then the prep's [Kpad][128] zero-padded copy; the hi-only pass's
    // uncertified rows go straight to the caller's exact pass (no LIST form)
    int rows = 0;
    const double* X64 = nullptr;
    int d = 128;
    const double* Cd = nullptr;                  // general rows, cosine: the caller's [K][d] centroids
    // K > 256 on the persistent form: passes over 256-centroid slices carry each
    // lane's (best, runner-up, tile) in part[] (32 B per point)
    void* part = nullptr;
    int64_t part_bytes = 0;
    // hi-only form (euclidean): fused_hi_kernel, then the 3-product LIST form on
    // its uncertified rows (list2 / seg_counts2: [list_cap] / [2 * seg_cap]);
    // out: refined = rows the hi-only pass left to the 3-product form (device)
    bool hi = false;
    int32_t* list2 = nullptr;
    int32_t* seg_counts2 = nullptr;
    unsigned long long* refined = nullptr;
    // hi-only cosine: the LIST form's declined winner distances go to a second
    // fix-up list (hfix2: [list_cap] entries after the first); out: the lists
    // for cos_fix_seg, (list, segment counts) pairs
    unsigned long long* hfix2 = nullptr;
    // hi-only cosine: the hi-only pass's declined winner distances ([list_cap]
    // entries, counts in cfix_counts[2b + 1], total in cfix_count)
    unsigned long long* cfix = nullptr;
    int32_t* cfix_counts = nullptr;
    unsigned long long* cfix_count = nullptr;
    int ncos_lists = 0;
    const unsigned long long* cos_list[2] = {nullptr, nullptr};
    const int32_t* cos_counts[2] = {nullptr, nullptr};
    // out: the list of rows still uncertified for the exact pass
    const int32_t* final_list = nullptr;
    const int32_t* final_counts = nullptr;
};
constexpr int64_t FUSED_PART_BYTES_PER_ROW = 32;
// List capacity the persistent form may need beyond N entries (grid <= 1024 blocks).
constexpr int64_t FUSED_LIST_SLACK = 32 + 1024 * 12 * 32;
constexpr int FUSED_MAX_SEGS = 1024;
int launch_fused_prep(hipStream_t s, const double* C, int K, int Kpad, _Float16* Ch, _Float16* Cl, float* cnh,
                      float* cbound, int metric = 0, double* nbv = nullptr, float* C32 = nullptr,
                      float* rn32 = nullptr, int d = 128, double* C64p = nullptr);
int launch_fused(hipStream_t s, bool hash, FusedLaunch& f);
// out[i] = sum_j pow(x_ij, 2) in j order (glibc's pow, gpow2.h), fp64 rows
int launch_row_sumsq(hipStream_t s, const double* X, int64_t N, int d, double* out);
// Winners listed by the fused kernels for their distance alone (segment b:
// list[b * seg_rows ..], count counts[2b + 1]): metric 1 the soft-x87 cosine,
// metric 0 the euclidean chain with glibc's pow(x, 2) (gpow2.h).
int launch_cos_fix_seg(hipStream_t s, Pts X, int d, const double* C, int nlists, const unsigned long long* const* lists,
                       const int32_t* const* counts, int64_t seg_rows, int nseg, const int32_t* assign, double* dist,
                       int metric, const double* xn2 = nullptr, const double* nbv = nullptr);

// Range assignment (range.hip).
int launch_range_radius(hipStream_t s, const double* C, int K, int d, int metric, double* r0,
                        unsigned long long* tmp);
int launch_range_pairs(hipStream_t s, const int64_t* comb_ptr, const int32_t* comb_idx, int K, int32_t* rows,
                       int32_t* cents);
int launch_range_init(hipStream_t s, int64_t N, int32_t* assign, double* dist);
int launch_range_pass(hipStream_t s, Pts X, int d, const double* C, int K, int metric, const int32_t* key,
                      const int64_t* vptr, const int32_t* cents, double* cache, int8_t* cached, int64_t N,
                      const double* r0, int64_t pass, int32_t* assign, double* dist, unsigned long long* count);
int launch_range_unassigned(hipStream_t s, const int32_t* assign, int64_t N, int32_t* list,
                            unsigned long long* count);
// Xr: rows of the same element type as X
int launch_range_gather(hipStream_t s, Pts X, int d, const int32_t* list, int64_t M, void* Xr);
int launch_range_scatter(hipStream_t s, const int32_t* list, int64_t M, const int32_t* ar, const double* dr,
                         int32_t* assign, double* dist);

// Silhouette (silhouette.hip).
int launch_sil_near(hipStream_t s, const double* C, int K, int d, int metric, int32_t* near);
int launch_sil_points(hipStream_t s, Pts X, int d, int metric, const int32_t* rows, const int64_t* crow,
                      const int32_t* assign, const int32_t* near, int64_t N, double* s_out, bool exsq = false);
int launch_sil_sum(hipStream_t s, const double* sv, const int32_t* rows, const int64_t* crow, int K, int64_t N,
                   double* raw, double* out);

// Synthetic data.
int launch_synth(hipStream_t s, uint64_t seed, int64_t row0, int64_t rows, int d, float* X, int kind = 0);

}  // namespace lshkm
