/*
 * lshkm_oracle.h — CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline). The product (crypto-recommendation_amd/) never
 * links or calls it.
 *
 * Pinned by: the tests/golden fixtures, produced by oracle/_ref/ref_harness — the
 * reference's own code compiled from /root/reference (see oracle/Makefile,
 * tests/golden/make_golden.py).
 *
 * Rows are fp64, as the reference holds them (CustVector<double>,
 * vector_reader.hpp:54-85): fp32 data widens exactly, general doubles (the
 * product's `_f64` entry points) are taken as they are. Centroids are fp64.
 */
#ifndef LSHKM_ORACLE_H
#define LSHKM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- libstdc++-11 <random> restatement (minstd_rand0 = default_random_engine) */
uint32_t or_minstd_seed(uint64_t seed);
uint32_t or_minstd_next(uint32_t* state);
int      or_uniform_int(uint32_t* state, int a, int b);

/* ---- parameter generation in the reference's draw order; each returns the
 * engine state after the last draw. */
uint32_t or_gen_lsh_euclid(uint64_t seed, int L, int k, int d, float w,
                           float* V /*[L][k][d]*/, float* t /*[L][k]*/, int32_t* r /*[L][k]*/);
uint32_t or_gen_lsh_cosine(uint64_t seed, int L, int k, int d, double* R /*[L][k][d]*/);
uint32_t or_gen_cube_euclid(uint64_t seed, int k, int d, float w, float* V /*[k][d]*/, float* t /*[k]*/);
uint32_t or_gen_cube_cosine(uint64_t seed, int k, int d, double* R /*[k][d]*/);

/* ---- hash families */
int32_t or_euclid_h(const float* v, const double* x, int d, float t, float w);
int32_t or_cosine_h(const double* r, const double* x, int d);
void or_lsh_hash_euclid(int64_t N, int d, int L, int k, const double* X,
                        const float* V, const float* t, float w, const int32_t* r, int64_t nb,
                        int32_t* tuples /*[N][L][k]*/, int32_t* phi /*[N][L]*/, int32_t* bucket /*[N][L]*/);
void or_lsh_hash_cosine(int64_t N, int d, int L, int k, const double* X, const double* R,
                        int32_t* g /*[N][L]*/);

/* ---- hashtables: stable bucket CSR (insertion order = row order) */
void or_bucket_csr(int64_t N, int L, int64_t nb, const int32_t* bucket /*[N][L]*/,
                   int64_t* row_ptr /*[L][nb+1]*/, int32_t* idx /*[L][N]*/);

/* ---- LSH query: union of L buckets (filtered by k-tuple if tuples != NULL),
 * deduped and index-sorted. Returns the count written (cap = out capacity). */
int64_t or_lsh_query(int64_t N, int L, int k, int64_t nb,
                     const int32_t* tuples /*[N][L][k] or NULL*/, const int64_t* row_ptr,
                     const int32_t* idx, const int32_t* q_tuple /*[L][k] or NULL*/,
                     const int32_t* q_bucket /*[L]*/, int32_t* out, int64_t cap);

/* ---- hypercube */
void or_cube_h(int64_t N, int d, int k, const double* X, const float* V, const float* t, float w,
               int32_t* h /*[N][k]*/);
/* Lazy F coins (euclidean_f_gen.hpp:65-79). memo is [k][hspan] (entries -1 =
 * unseen) indexed by h - hmin. Draws happen in (row, f) order. Returns the
 * number of draws; updates *state. Fails (-1) if an h is outside the span. */
int64_t or_cube_coins(int64_t N, int k, const int32_t* h, int32_t hmin, int32_t hspan,
                      int32_t* memo, uint32_t* state, int32_t* vertex /*[N]*/);
void or_cube_cosine(int64_t N, int d, int k, const double* X, const double* R, int32_t* vertex);
/* Probe sequence of get_hypercube_combined_buckets (lsh_cube.hpp:139-177):
 * writes at most cap vertices (main bucket first). Returns the count. */
int64_t or_cube_probe_seq(int32_t vertex, int probes, int k, int32_t* out, int64_t cap);

/* ---- Lloyd assignment (assignment.hpp:54-80). metric 0 = euclidean, 1 = cosine.
 * src_rows[K] (or NULL): dataset row of each centroid (-1 = none) for the
 * centroid override at assignment.hpp:77-78. */
void or_lloyd_assign(int64_t N, int d, int K, const double* X, const double* C, int metric,
                     const int32_t* src_rows, int32_t* assign, double* dist);
double or_euclid_dist(const double* x, const double* c, int d);

/* ---- k-means update (update.hpp:37-86). Returns 1 = continue (centers move),
 * 0 = converged. C_new always written; counts[K] written. */
int or_kmeans_update(int64_t N, int d, int K, const double* X, const int32_t* assign,
                     const double* C_old, int metric, double min_dist, double* C_new, int64_t* counts);

/* ---- range assignment (assignment.hpp:108-217): combined buckets per
 * centroid as a CSR, key[K] = distance-cache key per centroid (NULL = all
 * distinct). Returns the number of passes. */
int or_range_assign(int64_t N, int d, int K, const double* X, const double* C, int metric,
                    const int64_t* comb_ptr, const int32_t* comb_idx, const int32_t* key,
                    const int32_t* src_rows, int32_t* assign, double* dist);

/* ---- silhouette_cluster (silhouette.hpp:31-144): out[K+1], s[N] (or NULL) */
void or_silhouette(int64_t N, int d, int K, const double* X, const int32_t* assign, const double* C, int metric,
                   double* out, double* s);

/* ---- initialization (initialization.hpp:39-156): the chosen dataset rows */
void or_rand_selection(uint64_t seed, int64_t N, int K, int32_t* rows);
void or_kmeans_pp(int64_t N, int d, int K, const double* X, int metric, uint64_t seed, int32_t* rows);

/* ---- recommendation (crypto_rec.hpp:213-345) */
void or_p_closest(int d, const double* X, int64_t nq, const double* U, const int64_t* cand_ptr,
                  const int32_t* cand_idx, int P, int32_t* out_idx, double* out_sim, int32_t* out_cnt);
void or_top_n_recom(int d, const double* X, const double* x_mean, int64_t nq, const double* U,
                    const double* u_mean, const int64_t* unk_ptr, const int32_t* unk_idx, const int32_t* nb_idx,
                    const double* nb_sim, const int32_t* nb_cnt, int P, int N, int32_t* out);
/* the 3-argument get_top_N_recom over each user's whole cluster (:327-345) */
void or_cluster_top_n(int d, const double* X, const double* x_mean, const int64_t* crow, const int32_t* crows,
                      int64_t nq, const double* U, const double* u_mean, const int32_t* ucl,
                      const int64_t* unk_ptr, const int32_t* unk_idx, int N, int32_t* out);

/* ---- synthetic points (include/lshkm_synth.h) */
void or_synth(uint64_t seed, int64_t row0, int64_t rows, int d, float* out);
void or_synth_normal(uint64_t seed, int64_t row0, int64_t rows, int d, float* out);

#ifdef __cplusplus
}
#endif
#endif
