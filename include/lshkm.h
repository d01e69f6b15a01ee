/*
 * lshkm.h — C ABI of the MI355X (gfx950) LSH / hypercube / k-means hot path.
 *
 * Drop-in boundary for the reference's header-template interface
 * (paths relative to the reference root):
 *   create_LSH_hashtables            lib/lsh_cube.hpp:44-74
 *   get_LSH_combined_buckets         lib/lsh_cube.hpp:77-90
 *   get_LSH_filtered_combined_buckets lib/lsh_cube.hpp:93-106
 *   create_hypercube                 lib/lsh_cube.hpp:108-136
 *   get_hypercube_combined_buckets   lib/lsh_cube.hpp:139-177
 *   lloyds_assignment                lib/clustering_phases/assignment.hpp:54-80
 *   k_means                          lib/clustering_phases/update.hpp:37-86
 *   lsh_/cube_range_assignment       lib/clustering_phases/assignment.hpp:108-217
 *   silhouette_cluster               lib/clustering_phases/silhouette.hpp:31-144
 *   VectorReader<double>::read       lib/in_out/vector_reader.hpp:54-85
 *   file_to_args + ArgParser, get_config  lib/utils.cpp:53-69, lib/in_out/arg_parser.cpp, main.cpp:512-554
 *   HashGenerator plugin ABI         lib/generators/hash_generator.hpp:19-31
 *   CustHashtable::getBucketFromIndex / getHash lib/data_structures/cust_hashtable.hpp:116-125
 *
 * Conventions
 *   - Every function returns 0 on success or a negative LSHKM_ERR_* code;
 *     lshkm_last_error() then describes it (thread-local).
 *   - "_dev" pointers are device (HBM) pointers, "_host" pointers host memory.
 *     Sizes are explicit. Device outputs are written asynchronously on the
 *     context's stream; call lshkm_ctx_sync() before reading them on the host.
 *   - Points are N x d row-major rows of fp32 (the synthetic / proj-2 values
 *     are fp32-representable: the tuned storage) or of fp64: every entry
 *     point that reads dataset rows has a `_f64` twin taking `const double*`
 *     rows with the same results contract (the reference's CustVector<double>
 *     holds general doubles, e.g. the recommender's user vectors,
 *     crypto_rec.hpp:78-140). Centroids are fp64 rows, K x d.
 *   - Bit-exact with the reference: tuples, phi, bucket IDs, bucket member
 *     order, query results, hypercube vertices, probe order, cluster IDs,
 *     k-means centers and counts, chosen k-means++ rows, recommendations.
 *   - Distances (the `dist` output of the Lloyd / hash+assign entry points)
 *     follow the context's distance mode (lshkm_ctx_set_dist_mode):
 *       LSHKM_DIST_CERTIFIED (the default): euclidean winner distances may come
 *         from a certified f32 evaluation, within 2^-20 relative of the
 *         reference's fp64 value (the north star's tolerance is 1e-5); a row
 *         whose bound fails gets the reference-order chain. Zero, inf and NaN
 *         distances are reproduced bit for bit. Cluster IDs are unaffected.
 *       LSHKM_DIST_EXACT: every distance is the reference's sequential fp64
 *         chain sqrt(sum_j pow(x_j - c_j, 2)), j ascending, bit for bit --
 *         for dataset-row centroids and for general fp64 centroids after an
 *         update alike.
 *     Cosine distances, range-assignment distances, silhouettes, similarities
 *     and every other output are exact-order in both modes.
 *   - Every square the reference takes is glibc's pow(x, 2) (cust_vector.hpp:
 *     132, 149-150, 168-169), which is not x*x for ~0.085 % of general doubles
 *     (and for many exact ties): the device evaluates glibc 2.35's own
 *     algorithm (the x86-64 __pow_fma variant, csrc/gpow2.h) wherever x*x is
 *     not provably the same value. lshkm_pow_selfcheck() compares that
 *     restatement with the running process's pow; lshkm_ctx_create runs it
 *     once per process and refuses (LSHKM_ERR_UNSUPPORTED, see
 *     lshkm_last_error) on a host whose pow differs, since the reference's
 *     own results on that host could not be reproduced bit for bit.
 *   - One handle per thread; calls on a handle are serialised on its stream.
 */
#ifndef LSHKM_H
#define LSHKM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSHKM_OK 0
#define LSHKM_ERR_ARG (-1)
#define LSHKM_ERR_HIP (-2)
#define LSHKM_ERR_NOMEM (-3)
#define LSHKM_ERR_UNSUPPORTED (-4)
#define LSHKM_ERR_STATE (-5)

#define LSHKM_METRIC_EUCLIDEAN 0
#define LSHKM_METRIC_COSINE 1

#define LSHKM_DIST_CERTIFIED 0   /* euclidean winner distances within 2^-20 relative (default) */
#define LSHKM_DIST_EXACT 1       /* the reference's fp64 chain for every distance */

typedef struct lshkm_ctx_s* lshkm_ctx;
typedef struct lshkm_lsh_s* lshkm_lsh;
typedef struct lshkm_cube_s* lshkm_cube;
typedef struct lshkm_vectors_s* lshkm_vectors;

/* ------------------------------------------------------------------ context */
const char* lshkm_last_error(void);
const char* lshkm_version(void);
/* pow(x, 2) as the reference computes it (glibc's pow, cust_vector.hpp:132):
 * out_dev[i] for x_dev[i], i < n, on the device (csrc/gpow2.h). */
int lshkm_pow2(lshkm_ctx ctx, const double* x_dev, int64_t n, double* out_dev);
/* Host-only (no GPU): compares the device's restatement of glibc's pow(x, 2)
 * (the same code, compiled for the host) with this process's own pow on a
 * fixed set of inputs whose squares lie near rounding midpoints (the inputs
 * that tell pow from x*x) plus exact ties and special ranges; *mismatches_host
 * = how many differ (0 when the process's libm is the one the restatement
 * follows), *tested_host = inputs tried. */
int lshkm_pow_selfcheck(int64_t* mismatches_host, int64_t* tested_host);
/* A context on `device` (gfx950). Fails with LSHKM_ERR_UNSUPPORTED, before any
 * device work, when this process's pow(x, 2) differs from the restatement
 * (the pow contract above; checked once per process). */
int lshkm_ctx_create(int device, lshkm_ctx* out);
/* Run on a caller-owned hipStream_t (e.g. torch's current stream), used
 * verbatim: NULL is the default (null) stream. A new context uses its own stream. */
int lshkm_ctx_set_stream(lshkm_ctx ctx, void* hip_stream);
/* Distance contract of the context (see Conventions): LSHKM_DIST_CERTIFIED
 * (the default of a new context) or LSHKM_DIST_EXACT (the reference's
 * euclideanDistance, cust_vector.hpp:124-136, for every row; a few percent
 * slower at d = 128). The context's mode alone decides (no environment
 * override in this library). */
int lshkm_ctx_set_dist_mode(lshkm_ctx ctx, int mode);
int lshkm_ctx_get_dist_mode(lshkm_ctx ctx, int* mode_host);
int lshkm_ctx_sync(lshkm_ctx ctx);
int lshkm_ctx_destroy(lshkm_ctx ctx);
/* Device memory for callers without HIP headers (the C++ shim
 * include/lshkm_compat.hpp, cgo/JNI bindings). Copies are ordered on the
 * context's stream and complete before return; free waits for the stream. */
int lshkm_dev_alloc(lshkm_ctx ctx, int64_t bytes, void** out_dev);
int lshkm_dev_free(lshkm_ctx ctx, void* p_dev);
int lshkm_memcpy_h2d(lshkm_ctx ctx, void* dst_dev, const void* src_host, int64_t bytes);
int lshkm_memcpy_d2h(lshkm_ctx ctx, void* dst_host, const void* src_dev, int64_t bytes);
/* Counters: 0 = hash values resolved by the exact soft-x87 path,
 * 1 = points whose argmin needed the exact all-centroid pass,
 * 2 = k-means++ prefix-sum chunks walked, 3 = of which summed element by element,
 * 4 = cosine Lloyd winner distances the certified fast form declined (soft-x87 chain),
 * 5 = rows the hi-only fused pass (one f16 product per score) left to the 3-product form,
 * 6 = rows the fused pass listed for the hash fix-up,
 * 7 = clustering-recommender similarities decided by the x87 chain (lshkm_cluster_top_n),
 * 8 = euclidean winner distances (LSHKM_DIST_EXACT, hi-only pass) whose chain met an
 *     inexact square and were redone with glibc's pow(x, 2) (gpow2.h),
 * 9 = k-means (cluster, dim) sums of fp32 rows whose never-rounds test failed,
 *     i.e. that took a rounding-aware chain instead of plain fp64 adds. */
int lshkm_get_stat(lshkm_ctx ctx, int which, int64_t* value_host);
int lshkm_reset_stats(lshkm_ctx ctx);
/* HIP-event timing of the dominant kernel launch (the fused hash+assign kernel)
 * on the context's stream; lshkm_last_kernel_ms waits for and returns the last one. */
int lshkm_ctx_enable_timing(lshkm_ctx ctx, int on);
int lshkm_last_kernel_ms(lshkm_ctx ctx, float* ms_host);

/* ------------------------------------------- parameter generation (host)
 * std::default_random_engine seeded with `seed`, draws in the reference's
 * order; *rng_state_host receives the engine state after the last draw.
 * Replaces the generator constructors:
 *   EuclideanPhiGen  lib/generators/euclidean_phi_gen.hpp:59-71 (via euclidean_h_gen.hpp:56-69)
 *   CosineGGen       lib/generators/cosine_g_gen.hpp:48-52     (via cosine_h_gen.hpp:53-60)
 *   create_hypercube lib/lsh_cube.hpp:112-126                  (EuclideanFGen / CosineHGen) */
int lshkm_params_lsh_euclidean(uint64_t seed, int L, int k, int d, float w,
                               float* V_host /*[L][k][d]*/, float* t_host /*[L][k]*/,
                               int32_t* r_host /*[L][k]*/, uint32_t* rng_state_host);
int lshkm_params_lsh_cosine(uint64_t seed, int L, int k, int d, double* R_host /*[L][k][d]*/,
                            uint32_t* rng_state_host);
int lshkm_params_cube_euclidean(uint64_t seed, int k, int d, float w, float* V_host /*[k][d]*/,
                                float* t_host /*[k]*/, uint32_t* rng_state_host);
int lshkm_params_cube_cosine(uint64_t seed, int k, int d, double* R_host /*[k][d]*/,
                             uint32_t* rng_state_host);

/* ---------------------------------------------------------------- LSH index
 * create_LSH_hashtables (lsh_cube.hpp:44-74): metric EUCLIDEAN uses
 * EuclideanPhiGen with nb = N / lsh_bucket_div buckets; COSINE uses CosineGGen
 * with 2^k buckets (nb ignored). Parameters are copied to the device.
 * V/t/r for EUCLIDEAN, R for COSINE (the other may be NULL). */
int lshkm_lsh_create(lshkm_ctx ctx, int metric, int d, int k, int L, int64_t nb, float w,
                     const float* V_host, const float* t_host, const int32_t* r_host,
                     const double* R_host, lshkm_lsh* out);
int lshkm_lsh_destroy(lshkm_lsh lsh);
/* Hash a batch without inserting: EuclideanPhiGen::generate
 * (euclidean_phi_gen.hpp:77-92) + mod(phi, nb) (cust_hashtable.hpp:68).
 * tuples_dev [N][L][k] (EUCLIDEAN only), phi_dev [N][L], bucket_dev [N][L];
 * any output may be NULL. For COSINE phi == bucket == g. */
int lshkm_lsh_hash(lshkm_lsh lsh, const float* X_dev, int64_t N, int32_t* tuples_dev,
                   int32_t* phi_dev, int32_t* bucket_dev);
int lshkm_lsh_hash_f64(lshkm_lsh lsh, const double* X_dev, int64_t N, int32_t* tuples_dev,
                       int32_t* phi_dev, int32_t* bucket_dev);
/* Insert all N rows (create_LSH_hashtables' insert loop, lsh_cube.hpp:69-70):
 * hashes, then a stable bucket scatter (member order = row order,
 * vector_bucket.hpp:41-44). The dataset rows and their tuples stay
 * device-resident in the handle (X_dev must stay valid for queries that use
 * alias rows only through their tuples; it is not read again). */
int lshkm_lsh_build(lshkm_lsh lsh, const float* X_dev, int64_t N);
int lshkm_lsh_build_f64(lshkm_lsh lsh, const double* X_dev, int64_t N);
/* Bucket contents of one table (getBucketFromIndex, cust_hashtable.hpp:116-119):
 * row_ptr_host [nb+1], idx_host [N]. */
int lshkm_lsh_get_buckets(lshkm_lsh lsh, int table, int64_t* row_ptr_host, int32_t* idx_host);
/* Device views of the built index (valid until destroy/rebuild). */
int lshkm_lsh_device_views(lshkm_lsh lsh, const int64_t** row_ptr_dev /*[L][nb+1]*/,
                           const int32_t** idx_dev /*[L][N]*/, const int32_t** tuples_dev /*[N][L][k]*/,
                           const int32_t** bucket_dev /*[N][L]*/);
/* Batched queries (get_LSH_filtered_combined_buckets, lsh_cube.hpp:93-106,
 * or get_LSH_combined_buckets :77-90 when filtered == 0). Output per query:
 * the deduplicated union of its L buckets, ascending row index (std::set
 * order). alias_rows_dev[q] >= 0 says "query q has the ID of dataset row r":
 * the reference's first-write-wins ID map (euclidean_phi_gen.hpp:94) then
 * filters with row r's tuple. May be NULL.
 * Two-phase: out_ptr_dev [nq+1] always written (prefix offsets); rows are
 * written to out_idx_dev only if total <= out_cap. *total_host = total rows.
 * A filling call (out_idx_dev != NULL) right after a sizing call (NULL) with
 * the same Q_dev, nq, alias_rows_dev, filtered and out_ptr_dev buffer -- and no
 * other call on the context's workspace in between -- reuses the sizing call's
 * device state: the contents of Q, alias and out_ptr must not change between
 * the two calls. Any other filling call recomputes everything. */
int lshkm_lsh_query(lshkm_lsh lsh, const float* Q_dev, int64_t nq, const int32_t* alias_rows_dev,
                    int filtered, int64_t* out_ptr_dev, int32_t* out_idx_dev, int64_t out_cap,
                    int64_t* total_host);
int lshkm_lsh_query_f64(lshkm_lsh lsh, const double* Q_dev, int64_t nq, const int32_t* alias_rows_dev,
                        int filtered, int64_t* out_ptr_dev, int32_t* out_idx_dev, int64_t out_cap,
                        int64_t* total_host);

/* ---------------------------------------------------------------- hypercube
 * create_hypercube (lsh_cube.hpp:108-136): k EuclideanFGen (V,t,w + the lazy
 * coin engine state rng_state) or k CosineHGen (R); 2^k buckets. */
int lshkm_cube_create(lshkm_ctx ctx, int metric, int d, int k, float w, const float* V_host,
                      const float* t_host, const double* R_host, uint32_t rng_state, lshkm_cube* out);
int lshkm_cube_destroy(lshkm_cube cube);
/* Insert N rows: vertices (HypercubeGen::generate, hypercube_gen.hpp:63-73)
 * with EuclideanF coins drawn on first sight of each h in (row, f) order
 * (euclidean_f_gen.hpp:65-79), then the stable scatter into 2^k buckets. */
int lshkm_cube_build(lshkm_cube cube, const float* X_dev, int64_t N);
int lshkm_cube_build_f64(lshkm_cube cube, const double* X_dev, int64_t N);
/* Vertices of a query batch (getHash, cust_hashtable.hpp:122-125). Unseen h
 * values draw new coins in (query, f) order from the continued engine. */
int lshkm_cube_vertices(lshkm_cube cube, const float* Q_dev, int64_t nq, int32_t* vertex_dev);
int lshkm_cube_vertices_f64(lshkm_cube cube, const double* Q_dev, int64_t nq, int32_t* vertex_dev);
int lshkm_cube_get_buckets(lshkm_cube cube, int64_t* row_ptr_host /*[2^k+1]*/, int32_t* idx_host /*[N]*/);
/* get_hypercube_combined_buckets (lsh_cube.hpp:139-177): main bucket then
 * `probes` neighbours in get_num_hamming_dist_from order (utils.cpp:22-50),
 * probes == 1 skipping distance 1 as the reference does. Two-phase like
 * lshkm_lsh_query. */
int lshkm_cube_query(lshkm_cube cube, const float* Q_dev, int64_t nq, int probes,
                     int64_t* out_ptr_dev, int32_t* out_idx_dev, int64_t out_cap, int64_t* total_host);
int lshkm_cube_query_f64(lshkm_cube cube, const double* Q_dev, int64_t nq, int probes,
                         int64_t* out_ptr_dev, int32_t* out_idx_dev, int64_t out_cap, int64_t* total_host);
/* Sharded build of the euclidean cube (the coins of
 * euclidean_f_gen.hpp:65-79 must be drawn in GLOBAL first-occurrence order):
 * 1. each shard: lshkm_cube_unseen -> the (f, h) pairs of its rows that have
 *    no coin yet, with their first local row (row_host; add the shard's row0);
 *    if *count_host > cap nothing is copied and the call may be repeated;
 * 2. all-gather, keep each (f, h) at its smallest global (row * k + f), sort by
 *    it, and draw with lshkm_coins_draw (identical on every rank);
 * 3. each shard: lshkm_cube_import_coins (memo + the engine state after the
 *    draws), then lshkm_cube_build (no coin left to draw). */
int lshkm_cube_unseen(lshkm_cube cube, const float* X_dev, int64_t N, int32_t* f_host, int32_t* h_host,
                      int64_t* row_host, int64_t cap, int64_t* count_host);
int lshkm_cube_unseen_f64(lshkm_cube cube, const double* X_dev, int64_t N, int32_t* f_host, int32_t* h_host,
                          int64_t* row_host, int64_t cap, int64_t* count_host);
int lshkm_cube_import_coins(lshkm_cube cube, const int32_t* f_host, const int32_t* h_host, const int32_t* bit_host,
                            int64_t n, uint32_t rng_state);
/* Host draw of n coins in order from *rng_state (minstd_rand0 state, updated):
 * bit[i] = mod(h[i], uniform_int_distribution<int>(1, 2)). No device needed. */
int lshkm_coins_draw(uint32_t* rng_state, const int32_t* h_host, int64_t n, int32_t* bit_host);
/* Coin memo export: f_host/h_host/bit_host [cap]; *count_host = entries. */
int lshkm_cube_get_memo(lshkm_cube cube, int32_t* f_host, int32_t* h_host, int32_t* bit_host,
                        int64_t cap, int64_t* count_host, uint32_t* rng_state_host);

/* ------------------------------------------------------------------ k-means
 * lloyds_assignment (assignment.hpp:54-80): for each row the centroid with the
 * smallest distance (strict '<', first index wins), its fp64 distance, then
 * the centroid override: assign[src_rows[c]] = c, dist = 0 for c = 0..K-1
 * (src_rows_host may be NULL; entries outside [0, N) are ignored). */
int lshkm_lloyd_assign(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, const double* C_dev,
                       int K, int metric, const int32_t* src_rows_host, int32_t* assign_dev,
                       double* dist_dev);
int lshkm_lloyd_assign_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, const double* C_dev,
                           int K, int metric, const int32_t* src_rows_host, int32_t* assign_dev,
                           double* dist_dev);
/* The hot path in one pass over the points: LSH hashing of the rows
 * (EuclideanPhiGen::generate for every table, euclidean_phi_gen.hpp:77-92, and
 * the bucket index of cust_hashtable.hpp:68) and lloyds_assignment
 * (assignment.hpp:54-80) against C_dev. Outputs as lshkm_lsh_hash and
 * lshkm_lloyd_assign (tuples/phi/bucket may be NULL). Same results as the two
 * calls; one read of X when the index is euclidean with d = 128, L*k <= 32. */
int lshkm_hash_assign(lshkm_lsh lsh, const float* X_dev, int64_t N, const double* C_dev, int K,
                      const int32_t* src_rows_host, int32_t* tuples_dev, int32_t* phi_dev, int32_t* bucket_dev,
                      int32_t* assign_dev, double* dist_dev);
int lshkm_hash_assign_f64(lshkm_lsh lsh, const double* X_dev, int64_t N, const double* C_dev, int K,
                          const int32_t* src_rows_host, int32_t* tuples_dev, int32_t* phi_dev, int32_t* bucket_dev,
                          int32_t* assign_dev, double* dist_dev);
/* The same with the assignment metric chosen (lshkm_hash_assign is euclidean
 * Lloyd): main.cpp's cosine flow (main.cpp:150-160, 196) hashes with the
 * cosine family and clusters with cosineDistance. One read of X when the index
 * metric equals the assignment metric, d = 128, L*k <= 32 (cosine: k = 4). */
int lshkm_hash_assign_metric(lshkm_lsh lsh, const float* X_dev, int64_t N, const double* C_dev, int K, int metric,
                             const int32_t* src_rows_host, int32_t* tuples_dev, int32_t* phi_dev, int32_t* bucket_dev,
                             int32_t* assign_dev, double* dist_dev);
int lshkm_hash_assign_metric_f64(lshkm_lsh lsh, const double* X_dev, int64_t N, const double* C_dev, int K,
                                 int metric, const int32_t* src_rows_host, int32_t* tuples_dev, int32_t* phi_dev,
                                 int32_t* bucket_dev, int32_t* assign_dev, double* dist_dev);
/* k_means (update.hpp:37-86): exact-order per-cluster fp64 sums in row order,
 * divided by the count unless empty; *cont_host = 1 iff some center moved
 * more than min_dist. C_new_dev [K][d], counts_dev [K] (may be NULL). */
int lshkm_kmeans_update(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, const int32_t* assign_dev,
                        const double* C_old_dev, int K, int metric, double min_dist,
                        double* C_new_dev, int64_t* counts_dev, int* cont_host);
int lshkm_kmeans_update_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, const int32_t* assign_dev,
                            const double* C_old_dev, int K, int metric, double min_dist,
                            double* C_new_dev, int64_t* counts_dev, int* cont_host);
/* Sharded update (fast mode): per-shard exact-order sums, no division.
 * sums_dev [K][d], counts_dev [K]. Combine across ranks with an all-reduce,
 * then lshkm_kmeans_finalize. */
int lshkm_kmeans_partial(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, const int32_t* assign_dev,
                         int K, double* sums_dev, int64_t* counts_dev);
int lshkm_kmeans_partial_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, const int32_t* assign_dev,
                             int K, double* sums_dev, int64_t* counts_dev);
/* lshkm_kmeans_partial over the cluster CSR lshkm_clusters returned for the
 * same assignment (crow_dev [K+1], rows_dev [N]): the same sums without a
 * second sort when the caller needs the CSR anyway (the C5 iteration's
 * recommend step, main.cpp:261 over separate_clusters_from_input). */
int lshkm_kmeans_partial_csr(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, const int64_t* crow_dev,
                             const int32_t* rows_dev, int K, double* sums_dev, int64_t* counts_dev);
int lshkm_kmeans_partial_csr_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, const int64_t* crow_dev,
                                 const int32_t* rows_dev, int K, double* sums_dev, int64_t* counts_dev);
/* Sharded update (exact mode): the per-(c, j) chains continue from
 * carry_sums_dev / carry_counts_dev (the previous shard's result, or NULL for
 * the first shard), so passing the carry shard to shard in row order gives the
 * reference's single sequential sum (update.hpp:45-58) bit for bit. */
int lshkm_kmeans_partial_carry(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, const int32_t* assign_dev,
                               int K, const double* carry_sums_dev, const int64_t* carry_counts_dev,
                               double* sums_dev, int64_t* counts_dev);
int lshkm_kmeans_partial_carry_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d,
                                   const int32_t* assign_dev, int K, const double* carry_sums_dev,
                                   const int64_t* carry_counts_dev, double* sums_dev, int64_t* counts_dev);
/* Sharded update, bit-exact at all-reduce cost (the reference's
 * one sequential chain per (c, j), update.hpp:45-58, over row shards in rank
 * order). crow_dev / rows_dev: this rank's cluster CSR (lshkm_clusters).
 *  1. lshkm_kmeans_shard_begin: this rank's per-(c, j) partial sums (any
 *     order) sums_dev [K][d], the sums of |x| asum_dev [K][d], qt_dev [2][K][d]
 *     int32 (the lowest set-bit exponent of the values, then minus the top
 *     bit position), counts_dev [K].
 *  2. exchange: all-gather sums_dev in rank order into gathered [world][K][d];
 *     all-reduce asum_dev and counts_dev (SUM) and qt_dev (MIN).
 *  3. lshkm_kmeans_shard_certify (identical on every rank): per (c, j) the
 *     never-rounds test on the global values. Where it holds, every partial sum
 *     of any subset of the chain's values in any order is a double, so the
 *     total of the gathered partials IS the reference's chain: sums_out_dev.
 *     Elsewhere mask_dev [K][d] != 0: 2 for a chain of at most 32,768 values
 *     in all (one lane each in the chain phase), else 1 and flag_dev [K] has
 *     bit min(31, j / 64) set (segment records); start_dev [K][d] (may be
 *     NULL) = the chain's approximate value
 *     before this rank's rows (the lower ranks' partials); *n_flagged_host =
 *     the number of (c, j) masked (the same on every rank).
 *  4. only when *n_flagged_host > 0: lshkm_kmeans_shard_prepare (the lane
 *     list and the masked chains' binade-segment records from start_dev; all
 *     ranks at once), then
 *     in rank order lshkm_kmeans_shard_chain: the masked chains continued over
 *     this rank's rows from the previous rank's sums_out (carry_dev; NULL on
 *     rank 0), written into sums_dev where mask_dev is set; send sums_dev on.
 *     The last rank's sums_dev holds every chain's result: broadcast it.
 * ws_dev (prepare / chain; the same buffer for both): at least
 * lshkm_kmeans_shard_ws_bytes bytes, holding the records between the calls.
 * Then lshkm_kmeans_finalize on the totals and the all-reduced counts. One
 * rank (world 1) is the single-GPU update. sharding.kmeans_sums_sharded runs
 * the protocol over torch.distributed (RCCL on GPUs). */
int lshkm_kmeans_shard_begin(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, const int64_t* crow_dev,
                             const int32_t* rows_dev, int K, double* sums_dev, double* asum_dev, int32_t* qt_dev,
                             int64_t* counts_dev);
int lshkm_kmeans_shard_begin_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, const int64_t* crow_dev,
                                 const int32_t* rows_dev, int K, double* sums_dev, double* asum_dev, int32_t* qt_dev,
                                 int64_t* counts_dev);
int lshkm_kmeans_shard_certify(lshkm_ctx ctx, int K, int d, int world, int rank, const double* gathered_dev,
                               const double* asum_dev, const int32_t* qt_dev, const int64_t* counts_dev,
                               double* sums_out_dev, double* start_dev, int32_t* flag_dev, uint8_t* mask_dev,
                               int64_t* n_flagged_host);
int lshkm_kmeans_shard_ws_bytes(int64_t N, int K, int d, int64_t* bytes_host);
int lshkm_kmeans_shard_prepare(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, const int64_t* crow_dev,
                               const int32_t* rows_dev, int K, const double* start_dev, const int32_t* flag_dev,
                               const uint8_t* mask_dev, void* ws_dev, int64_t ws_bytes);
int lshkm_kmeans_shard_prepare_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, const int64_t* crow_dev,
                                   const int32_t* rows_dev, int K, const double* start_dev, const int32_t* flag_dev,
                                   const uint8_t* mask_dev, void* ws_dev, int64_t ws_bytes);
int lshkm_kmeans_shard_chain(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, const int64_t* crow_dev,
                             const int32_t* rows_dev, int K, const int32_t* flag_dev, const uint8_t* mask_dev,
                             const double* carry_dev, void* ws_dev, int64_t ws_bytes, double* sums_dev);
int lshkm_kmeans_shard_chain_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, const int64_t* crow_dev,
                                 const int32_t* rows_dev, int K, const int32_t* flag_dev, const uint8_t* mask_dev,
                                 const double* carry_dev, void* ws_dev, int64_t ws_bytes, double* sums_dev);
int lshkm_kmeans_finalize(lshkm_ctx ctx, const double* sums_dev, const int64_t* counts_dev, int K, int d,
                          const double* C_old_dev, int metric, double min_dist, double* C_new_dev,
                          int* cont_host);
/* separate_clusters_from_input (utils.hpp:150-158): the clusters' member lists
 * as a CSR, cluster c = rows_dev[crow_dev[c] .. crow_dev[c+1]) in row order
 * (the insertion order of the reference's per-cluster vectors). assign_dev
 * values must lie in [0, K) (what lshkm_lloyd_assign writes). crow_dev [K+1],
 * rows_dev [N]. */
int lshkm_clusters(lshkm_ctx ctx, const int32_t* assign_dev, int64_t N, int K, int64_t* crow_dev,
                   int32_t* rows_dev);

/* --------------------------------------------------------- range assignment
 * lsh_range_assignment / cube_range_assignment (assignment.hpp:108-145):
 * remove_clustering, range_assignment (:148-217) over the combined buckets of
 * the centroids, lloyds_for_remaining (:83-104) for the rows left unassigned,
 * then the centroid override (src_rows_host as in lshkm_lloyd_assign).
 * comb_ptr_dev [K+1] / comb_idx_dev: centroid i's combined bucket, in the
 * reference's order — what lshkm_lsh_query (filtered = 0) or lshkm_cube_query
 * returns for the centroid rows. Radius: find_min_vector_distance of the
 * centroids / 2 (utils.hpp:161-178), doubled after every centroid.
 * key_host [K] (may be NULL = all distinct): the reference caches distances by
 * "<centroid id>to<row id>" (:176-186), so centroids with the same ID share
 * entries (every "k_means_center" after k_means): give them equal keys.
 * *passes_host (may be NULL) = passes of the do-while loop. N < 2^31. */
int lshkm_range_assign(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, const double* C_dev, int K, int metric,
                       const int64_t* comb_ptr_dev, const int32_t* comb_idx_dev, const int32_t* key_host,
                       const int32_t* src_rows_host, int32_t* assign_dev, double* dist_dev, int* passes_host);
int lshkm_range_assign_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, const double* C_dev, int K,
                           int metric, const int64_t* comb_ptr_dev, const int32_t* comb_idx_dev,
                           const int32_t* key_host, const int32_t* src_rows_host, int32_t* assign_dev,
                           double* dist_dev, int* passes_host);

/* --------------------------------------------------------------- silhouette
 * silhouette_cluster (silhouette.hpp:31-80) over the clusters of `assign`
 * (separate_clusters_from_input, utils.hpp:150-158: members in row order)
 * with the K centroids C_dev (nearest other centroid = neighbour cluster).
 * out_host [K+1]: per-cluster mean s(i), then the overall mean; s_dev [N]
 * (may be NULL): silhouette_of_i of every row (:83-144). Exact distances in
 * the reference's order; NaNs as x86 produces them (empty cluster: 0/0). */
int lshkm_silhouette(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, const int32_t* assign_dev,
                     const double* C_dev, int K, int metric, double* out_host, double* s_dev);
int lshkm_silhouette_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, const int32_t* assign_dev,
                         const double* C_dev, int K, int metric, double* out_host, double* s_dev);

/* ----------------------------------------------------------- initialization
 * k_means_pp (initialization.hpp:71-156): the K dataset rows chosen as initial
 * centroids (centroids[i] = &input_vectors[rows_host[i]]), with
 * std::default_random_engine seeded with `seed` (the reference reads the
 * clock). D^2 seeding with the reference's exact distances, (min/max)^2
 * prefix sums in row order and its binary search. Assumes unique vector IDs
 * (the reference's distance cache is keyed by them). N < 2^31, d <= 4096. */
int lshkm_kmeans_pp(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, int K, int metric, uint64_t seed,
                    int32_t* rows_host);
int lshkm_kmeans_pp_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, int K, int metric, uint64_t seed,
                        int32_t* rows_host);
/* rand_selection (initialization.hpp:39-69): K distinct rows drawn uniformly,
 * redrawing on a repeat. Host only. 1 <= K <= N. */
int lshkm_rand_selection(uint64_t seed, int64_t N, int K, int32_t* rows_host);

/* ----------------------------------------------------------- recommendation
 * get_P_closest (crypto_rec.hpp:213-231) for nq users at once. User q's
 * neighbours are the dataset rows cand_idx_dev[cand_ptr_dev[q] ..
 * cand_ptr_dev[q+1]) in the order the reference's neighbour vector holds them
 * (ascending row: a query's output). Similarity = cosineSimilarity(neighbour,
 * user) (cust_vector.hpp:158-174); order = the reference's quicksort
 * (parallel_quickSort, :234-277, ties and NaNs included); first P kept.
 * Rows are fp64 (X_dev [N][d] neighbour pool, U_dev [nq][d] users).
 * out_idx_dev / out_sim_dev [nq][P] (-1 / 0 past the count), out_cnt_dev [nq]
 * = min(P, neighbours). Bit-exact on any doubles (the norms' squares are
 * glibc's pow(x, 2)). */
int lshkm_p_closest(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, const double* U_dev, int64_t nq,
                    const int64_t* cand_ptr_dev, const int32_t* cand_idx_dev, int P, int32_t* out_idx_dev,
                    double* out_sim_dev, int32_t* out_cnt_dev);
/* get_top_N_recom (crypto_rec.hpp:305-325) over lshkm_p_closest's lists:
 * predicted scores of each user's unknown indexes (get_predicted_user_sim,
 * :280-302; unk_* = CSR of the ascending unknown indexes, std::set order),
 * sorted by the same quicksort, first n_top (0-padded like vector::resize).
 * x_mean_dev [N] / u_mean_dev [nq]: getKnownMean of the rows / users.
 * out_dev [nq][n_top]. */
int lshkm_top_n_recom(lshkm_ctx ctx, const double* X_dev, const double* x_mean_dev, int64_t N, int d,
                      const double* u_mean_dev, int64_t nq, const int64_t* unk_ptr_dev, const int32_t* unk_idx_dev,
                      const int32_t* nb_idx_dev, const double* nb_sim_dev, const int32_t* nb_cnt_dev, int P,
                      int n_top, int32_t* out_dev);

/* get_top_N_recom(neighbors, user, N) -- the 3-argument overload
 * (crypto_rec.hpp:327-345) -- as the clustering recommenders call it:
 * main.cpp:260-269 (Part A: user q's own cluster) and :353-373 (Part B: the
 * cluster of the user's nearest centroid, i.e. lshkm_lloyd_assign of the users
 * without the override). User q's neighbours are the members of cluster
 * ucl_dev[q], crows_dev[crow_dev[c] .. crow_dev[c+1]) in member order (what
 * lshkm_clusters returns: separate_clusters_from_input, utils.hpp:150-158);
 * similarities = cosineSimilarity(member, user) in that order (x87-exact,
 * cust_vector.hpp:158-174); predictions = get_predicted_user_sim over all of
 * them (:280-306; x_mean_dev [N] / u_mean_dev [nq] = getKnownMean, unk_* = CSR
 * of each user's ascending unknown indexes, values in [0, d)); the reference's
 * quicksort of the predictions (:234-277, ties / NaNs included); out_dev
 * [nq][n_top] = the first n_top unknown indexes, 0-padded like vector::resize.
 * Users whose cluster is empty get -1 in every slot: main.cpp skips them
 * (:262, :366). A ucl outside [0, K) is LSHKM_ERR_ARG (the reference indexes
 * clusters[ucl] unchecked; the same holds for the sharded entry points below). X_dev [N][d] pool rows and U_dev [nq][d]
 * users share the element type (for Part A pass the same rows twice). Counter
 * 7 counts the similarities the x87 chain decided. Bit-exact on any rows (the
 * norms' squares are glibc's pow(x, 2)). */
int lshkm_cluster_top_n(lshkm_ctx ctx, const float* X_dev, const double* x_mean_dev, int64_t N, int d,
                        const int64_t* crow_dev, const int32_t* crows_dev, int K, const float* U_dev,
                        const double* u_mean_dev, int64_t nq, const int32_t* ucl_dev, const int64_t* unk_ptr_dev,
                        const int32_t* unk_idx_dev, int n_top, int32_t* out_dev);
int lshkm_cluster_top_n_f64(lshkm_ctx ctx, const double* X_dev, const double* x_mean_dev, int64_t N, int d,
                            const int64_t* crow_dev, const int32_t* crows_dev, int K, const double* U_dev,
                            const double* u_mean_dev, int64_t nq, const int32_t* ucl_dev, const int64_t* unk_ptr_dev,
                            const int32_t* unk_idx_dev, int n_top, int32_t* out_dev);

/* The same over row shards (the C5 recommend step): a cluster's
 * members lie on every rank, in row order = rank order, and
 * get_predicted_user_sim's sums (crypto_rec.hpp:285-303) run over them in that
 * order -- so the sums pass from rank to rank (point-to-point, like the exact
 * k-means carry). Every rank holds the same nq query users (U_dev rows,
 * u_mean, ucl = their global cluster IDs, the unknown lists) and the CSR of
 * its own rows' clusters (lshkm_clusters of its assignment: local row ids).
 * lshkm_cluster_sims: each user's similarities to this rank's members of its
 *   cluster, the bulk of the work and independent of the other ranks:
 *   soff_dev [nq+1] <- offsets; sims_dev [cap] <- the similarities in member
 *   order when *total_host <= cap (call with sims_dev = NULL to size).
 * lshkm_cluster_chain: the prediction sums continued over this rank's members
 *   from the previous rank's carry (carry_* all NULL on rank 0): carry_main /
 *   main_out [total unknown indexes] (per unknown index, unk_ptr order),
 *   carry_abs / abs_out and carry_cnt / cnt_out [nq] (sum |sim|, members so
 *   far); send the outputs to the next rank. The last rank passes out_dev
 *   [nq][n_top] instead (main_out etc. may be NULL): the predictions, the
 *   quicksort and the first n_top as lshkm_cluster_top_n, -1 for users whose
 *   cluster is empty on every rank. Chained over the ranks in row order this is
 *   lshkm_cluster_top_n over the concatenated rows, bit for bit. */
int lshkm_cluster_sims(lshkm_ctx ctx, const float* X_dev, int64_t N, int d, const int64_t* crow_dev,
                       const int32_t* crows_dev, int K, const float* U_dev, int64_t nq, const int32_t* ucl_dev,
                       const int64_t* unk_ptr_dev, int64_t* soff_dev, double* sims_dev, int64_t cap,
                       int64_t* total_host);
int lshkm_cluster_sims_f64(lshkm_ctx ctx, const double* X_dev, int64_t N, int d, const int64_t* crow_dev,
                           const int32_t* crows_dev, int K, const double* U_dev, int64_t nq, const int32_t* ucl_dev,
                           const int64_t* unk_ptr_dev, int64_t* soff_dev, double* sims_dev, int64_t cap,
                           int64_t* total_host);
int lshkm_cluster_chain(lshkm_ctx ctx, const float* X_dev, const double* x_mean_dev, int64_t N, int d,
                        const int64_t* crow_dev, const int32_t* crows_dev, int K, int64_t nq, const int32_t* ucl_dev,
                        const double* u_mean_dev, const int64_t* unk_ptr_dev, const int32_t* unk_idx_dev,
                        const int64_t* soff_dev, const double* sims_dev, const double* carry_main_dev,
                        const double* carry_abs_dev, const int64_t* carry_cnt_dev, double* main_out_dev,
                        double* abs_out_dev, int64_t* cnt_out_dev, int n_top, int32_t* out_dev);
int lshkm_cluster_chain_f64(lshkm_ctx ctx, const double* X_dev, const double* x_mean_dev, int64_t N, int d,
                            const int64_t* crow_dev, const int32_t* crows_dev, int K, int64_t nq,
                            const int32_t* ucl_dev, const double* u_mean_dev, const int64_t* unk_ptr_dev,
                            const int32_t* unk_idx_dev, const int64_t* soff_dev, const double* sims_dev,
                            const double* carry_main_dev, const double* carry_abs_dev, const int64_t* carry_cnt_dev,
                            double* main_out_dev, double* abs_out_dev, int64_t* cnt_out_dev, int n_top,
                            int32_t* out_dev);

/* The terms form of the same two phases (what sharding.recommend_sharded and
 * lshkm_cluster_top_n run): phase 1 also forms get_predicted_user_sim's terms
 * sim_i * (x_i[index] - mean_i) (crypto_rec.hpp:296) while the member rows are
 * on chip, so the rank-to-rank chain reads no rows.
 * lshkm_cluster_terms: soff_dev / toff_dev [nq+1] <- the offsets of each user's
 *   similarities (member order) and terms (member-major: toff[q] + i * m_q + e,
 *   m_q = the user's unknown indexes); sims_dev [cap] / terms_dev [tcap] filled when the totals
 *   (*total_host, *tterms_host) fit (NULL to size). Rows of d * sizeof(elem) a
 *   multiple of 8 B and at most 1016 B (else LSHKM_ERR_ARG: the form above).
 * lshkm_cluster_chain_terms: lshkm_cluster_chain from them (same carry and
 *   outputs). */
int lshkm_cluster_terms(lshkm_ctx ctx, const float* X_dev, const double* x_mean_dev, int64_t N, int d,
                        const int64_t* crow_dev, const int32_t* crows_dev, int K, const float* U_dev, int64_t nq,
                        const int32_t* ucl_dev, const int64_t* unk_ptr_dev, const int32_t* unk_idx_dev,
                        int64_t* soff_dev, int64_t* toff_dev, double* sims_dev, double* terms_dev, int64_t cap,
                        int64_t tcap, int64_t* total_host, int64_t* tterms_host);
int lshkm_cluster_terms_f64(lshkm_ctx ctx, const double* X_dev, const double* x_mean_dev, int64_t N, int d,
                            const int64_t* crow_dev, const int32_t* crows_dev, int K, const double* U_dev, int64_t nq,
                            const int32_t* ucl_dev, const int64_t* unk_ptr_dev, const int32_t* unk_idx_dev,
                            int64_t* soff_dev, int64_t* toff_dev, double* sims_dev, double* terms_dev, int64_t cap,
                            int64_t tcap, int64_t* total_host, int64_t* tterms_host);
int lshkm_cluster_chain_terms(lshkm_ctx ctx, int64_t nq, const double* u_mean_dev, const int64_t* unk_ptr_dev,
                              const int32_t* unk_idx_dev, const int64_t* soff_dev, const int64_t* toff_dev,
                              const double* sims_dev, const double* terms_dev, const double* carry_main_dev,
                              const double* carry_abs_dev, const int64_t* carry_cnt_dev, double* main_out_dev,
                              double* abs_out_dev, int64_t* cnt_out_dev, int n_top, int32_t* out_dev);

/* ------------------------------------------------------------ input formats
 * Host only (no device needed). VectorReader<double>::read
 * (vector_reader.hpp:54-85): lines 1..strt_line-1 kept as metadata, then one
 * vector per line: '\r' removed, ID = text before the first delimiter, values
 * = std::stod of each delimiter-separated token (getline semantics). A token
 * std::stod would throw on fails the call. threads <= 0: all hardware threads. */
int lshkm_vectors_read(const char* path, char delimiter, int strt_line, int threads, lshkm_vectors* out);
/* n rows, d = values of row 0, id_bytes = total ID length, ragged = rows of
 * different lengths, fp32_exact = every value is an fp32 value (the hot
 * path's storage contract), n_meta = metadata lines. Any pointer may be NULL. */
int lshkm_vectors_info(lshkm_vectors v, int64_t* n, int* d, int64_t* id_bytes, int* ragged, int* fp32_exact,
                       int* n_meta);
/* Row-major values: X64_host [n][d] and/or X32_host [n][d] (either may be NULL). */
int lshkm_vectors_values(lshkm_vectors v, double* X64_host, float* X32_host);
/* IDs: bytes_host [id_bytes] concatenated, offsets_host [n+1]. */
int lshkm_vectors_ids(lshkm_vectors v, char* bytes_host, int64_t* offsets_host);
/* getMetaLine(index) (vector_reader.hpp:91-96): "" past the saved lines. */
int lshkm_vectors_meta(lshkm_vectors v, int index, char* buf, int64_t cap, int64_t* len);
int lshkm_vectors_free(lshkm_vectors v);

/* cluster.conf: file_to_args(path, ' ') + ArgParser::getFlagValue — the token
 * after the first occurrence of key (*found = 0: absent, or last token). */
int lshkm_config_value(const char* path, const char* key, char* buf, int64_t cap, int* found);
/* get_config (main.cpp:512-554): the reference's defaults (main.cpp:50-63),
 * then every key present; csv_delimiter is an ASCII code, proj_2_csv_delimiter
 * the first character. Fails where the reference's stoi / stod would throw. */
typedef struct lshkm_config {
    char proj_2_input[1024];
    char proj_2_csv_delimiter;
    int proj_2_cluster_num;
    int cluster_num;
    int has_cluster_num;      /* 0: the reference would ask on stdin */
    int k, L, lsh_bucket_div;
    double euclidean_h_w;
    char csv_delimiter;
    int max_algo_iterations;
    double min_dist_kmeans;
    char lexicon_file[1024];
    char query_file[1024];
} lshkm_config;
int lshkm_config_load(const char* path, lshkm_config* out);

/* ------------------------------------------------------------ synthetic data */
/* include/lshkm_synth.h generator, rows [row0, row0+rows) into X_dev. */
int lshkm_synth(lshkm_ctx ctx, uint64_t seed, int64_t row0, int64_t rows, int d, float* X_dev);
/* The "normal" generator of include/lshkm_synth.h (Irwin-Hall(12), full fp32
 * mantissas; SURVEY.md §8d's N(0,1) rows), rows [row0, row0+rows) into X_dev. */
int lshkm_synth_normal(lshkm_ctx ctx, uint64_t seed, int64_t row0, int64_t rows, int d, float* X_dev);

#ifdef __cplusplus
}
#endif
#endif /* LSHKM_H */
