/*
 * lshkm_oracle.c — CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see lshkm_oracle.h). Every function cites the
 * reference file:line it restates (paths relative to the reference root).
 *
 * Numerics follow the reference exactly:
 *   - inner products accumulate in x87 long double, each product rounded to
 *     double first (cust_vector.hpp:105-121);
 *   - euclidean distances call the real libm pow(x, 2) (cust_vector.hpp:131-135);
 *     this file is built with -fno-builtin so gcc cannot fold pow(x,2) to x*x,
 *     matching the shipped -O0 build that calls pow@PLT;
 *   - no FMA contraction (-ffp-contract=off, no -mfma).
 */
#include "lshkm_oracle.h"
#include "../include/lshkm_synth.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ <random>
 * std::default_random_engine is minstd_rand0 (a=16807, m=2^31-1) in
 * libstdc++-11. seed(s): x = s mod m, 0 -> 1. */
uint32_t or_minstd_seed(uint64_t seed) {
    uint64_t x = seed % 2147483647ull;
    return (uint32_t)(x == 0 ? 1 : x);
}

uint32_t or_minstd_next(uint32_t* state) {
    *state = (uint32_t)(((uint64_t)*state * 16807ull) % 2147483647ull);
    return *state;
}

/* uniform_int_distribution<int>(a,b) downscaling path (the engine range
 * 2^31-2 is not a full 32/64-bit range): scale = urngrange / uerange,
 * reject ret >= uerange*scale, return ret/scale + a. */
int or_uniform_int(uint32_t* state, int a, int b) {
    const uint64_t urngrange = 2147483646ull - 1ull;
    const uint64_t urange = (uint64_t)((int64_t)b - (int64_t)a);
    if (urange == urngrange) return (int)((uint64_t)or_minstd_next(state) - 1ull + (uint64_t)(int64_t)a);
    if (urange > urngrange) return 0x80000000;  /* upscaling path: never used by the reference */
    const uint64_t uerange = urange + 1;
    const uint64_t scaling = urngrange / uerange;
    const uint64_t past = uerange * scaling;
    uint64_t ret;
    do { ret = (uint64_t)or_minstd_next(state) - 1ull; } while (ret >= past);
    return (int)(ret / scaling) + a;
}

/* generate_canonical<float, 24>: one engine call. tmp = float(1.0f * R) with
 * R = 2147483646.0L. */
static float canon_f(uint32_t* s) {
    const long double R = 2147483646.0L;
    float sum = (float)((uint64_t)or_minstd_next(s) - 1ull) * 1.0f;
    float tmp = (float)(1.0f * R);
    float ret = sum / tmp;
    if (ret >= 1.0f) ret = nextafterf(1.0f, 0.0f);
    return ret;
}

/* generate_canonical<double, 53>: two engine calls. */
static double canon_d(uint32_t* s) {
    const long double R = 2147483646.0L;
    double sum = 0.0, tmp = 1.0;
    for (int k = 0; k < 2; k++) {
        sum += (double)((uint64_t)or_minstd_next(s) - 1ull) * tmp;
        tmp = (double)(tmp * R);
    }
    double ret = sum / tmp;
    if (ret >= 1.0) ret = nextafter(1.0, 0.0);
    return ret;
}

/* normal_distribution<float>(0,1), Marsaglia polar, fresh object per call
 * site so the cached second variate is dropped at the end of a block. Note
 * the mixed float/double expression `float(2.0) * u - 1.0`. */
static void normals_f(uint32_t* s, int n, float* out) {
    int have = 0; float saved = 0.0f;
    for (int i = 0; i < n; i++) {
        float ret;
        if (have) { have = 0; ret = saved; }
        else {
            float x, y, r2;
            do {
                x = (float)((double)(2.0f * canon_f(s)) - 1.0);
                y = (float)((double)(2.0f * canon_f(s)) - 1.0);
                r2 = x * x + y * y;
            } while ((double)r2 > 1.0 || (double)r2 == 0.0);
            float mult = sqrtf(-2 * logf(r2) / r2);
            saved = x * mult; have = 1;
            ret = y * mult;
        }
        out[i] = ret * 1.0f + 0.0f;
    }
}

static void normals_d(uint32_t* s, int n, double* out) {
    int have = 0; double saved = 0.0;
    for (int i = 0; i < n; i++) {
        double ret;
        if (have) { have = 0; ret = saved; }
        else {
            double x, y, r2;
            do {
                x = 2.0 * canon_d(s) - 1.0;
                y = 2.0 * canon_d(s) - 1.0;
                r2 = x * x + y * y;
            } while (r2 > 1.0 || r2 == 0.0);
            double mult = sqrt(-2 * log(r2) / r2);
            saved = x * mult; have = 1;
            ret = y * mult;
        }
        out[i] = ret * 1.0 + 0.0;
    }
}

/* EuclideanHGen ctor (euclidean_h_gen.hpp:56-69): d normals, then t~U_float(0,w). */
static void gen_euclid_h(uint32_t* s, int d, float w, float* v, float* t) {
    normals_f(s, d, v);
    *t = canon_f(s) * (w - 0.0f) + 0.0f;
}

/* create_LSH_hashtables (lsh_cube.hpp:49-61) -> EuclideanPhiGen ctor
 * (euclidean_phi_gen.hpp:59-71): per table, per i: HGen then r_i~U_int[0,100]. */
uint32_t or_gen_lsh_euclid(uint64_t seed, int L, int k, int d, float w, float* V, float* t, int32_t* r) {
    uint32_t s = or_minstd_seed(seed);
    for (int l = 0; l < L; l++)
        for (int i = 0; i < k; i++) {
            size_t li = (size_t)l * k + i;
            gen_euclid_h(&s, d, w, V + li * d, t + li);
            r[li] = or_uniform_int(&s, 0, 100);
        }
    return s;
}

/* CosineGGen -> k x CosineHGen (cosine_g_gen.hpp:48-52, cosine_h_gen.hpp:53-60). */
uint32_t or_gen_lsh_cosine(uint64_t seed, int L, int k, int d, double* R) {
    uint32_t s = or_minstd_seed(seed);
    for (int l = 0; l < L; l++)
        for (int i = 0; i < k; i++) normals_d(&s, d, R + ((size_t)l * k + i) * d);
    return s;
}

/* create_hypercube (lsh_cube.hpp:112-126): k x EuclideanFGen (one HGen each). */
uint32_t or_gen_cube_euclid(uint64_t seed, int k, int d, float w, float* V, float* t) {
    uint32_t s = or_minstd_seed(seed);
    for (int i = 0; i < k; i++) gen_euclid_h(&s, d, w, V + (size_t)i * d, t + i);
    return s;
}

uint32_t or_gen_cube_cosine(uint64_t seed, int k, int d, double* R) {
    uint32_t s = or_minstd_seed(seed);
    for (int i = 0; i < k; i++) normals_d(&s, d, R + (size_t)i * d);
    return s;
}

/* ------------------------------------------------------------------- hashes */

/* EuclideanHGen::generate (euclidean_h_gen.hpp:73-76) over
 * CustVector<float>::inner_product<double> (cust_vector.hpp:105-121). */
int32_t or_euclid_h(const float* v, const double* x, int d, float t, float w) {
    long double acc = 0.0L;
    for (int j = 0; j < d; j++) {
        double p = (double)v[j] * (double)x[j];
        acc = acc + (long double)p;
    }
    return (int32_t)floorl((acc + (long double)t) / (long double)w);
}

/* CosineHGen::generate (cosine_h_gen.hpp:67-74). */
int32_t or_cosine_h(const double* r, const double* x, int d) {
    long double acc = 0.0L;
    for (int j = 0; j < d; j++) {
        double p = r[j] * (double)x[j];
        acc = acc + (long double)p;
    }
    return acc >= 0 ? 1 : 0;
}

/* mod(x, n) = (x % n + n) % n (utils.hpp:97-98) in its (long, int) form. */
static int32_t mod_long_int(long x, int n) { return (int32_t)((x % n + n) % n); }

/* EuclideanPhiGen::generate (euclidean_phi_gen.hpp:77-92) + insertVector's
 * mod(phi, buckets.size()) (cust_hashtable.hpp:68). M = int(pow(2,32)-5)
 * folds to 2147483647 under g++. */
void or_lsh_hash_euclid(int64_t N, int d, int L, int k, const double* X, const float* V,
                        const float* t, float w, const int32_t* r, int64_t nb,
                        int32_t* tuples, int32_t* phi, int32_t* bucket) {
    const int M = 2147483647;
#pragma omp parallel for schedule(static)
    for (int64_t n = 0; n < N; n++) {
        const double* x = X + n * d;
        for (int l = 0; l < L; l++) {
            uint32_t hash_num = 0;
            for (int i = 0; i < k; i++) {
                size_t li = (size_t)l * k + i;
                int hi = or_euclid_h(V + li * d, x, d, t[li], w);
                long temp = (long)(int)((unsigned)hi * (unsigned)r[li]);   /* int*int (no overflow at these ranges) */
                hash_num = hash_num + (uint32_t)mod_long_int(temp, M);
                if (tuples) tuples[(n * L + l) * k + i] = hi;
            }
            uint32_t p = (hash_num % (uint32_t)M + (uint32_t)M) % (uint32_t)M;
            if (phi) phi[n * L + l] = (int32_t)p;
            if (bucket) bucket[n * L + l] = (int32_t)((uint64_t)p % (uint64_t)nb);
        }
    }
}

/* CosineGGen::generate (cosine_g_gen.hpp:58-66): bits MSB-first; buckets 2^k
 * so mod(g, 2^k) = g (lsh_cube.hpp:65). */
void or_lsh_hash_cosine(int64_t N, int d, int L, int k, const double* X, const double* R, int32_t* g) {
#pragma omp parallel for schedule(static)
    for (int64_t n = 0; n < N; n++) {
        for (int l = 0; l < L; l++) {
            int h = 0;
            for (int i = 0; i < k; i++) h = (h << 1) + or_cosine_h(R + ((size_t)l * k + i) * d, X + n * d, d);
            g[n * L + l] = h;
        }
    }
}

/* VectorBucket insertion order (vector_bucket.hpp:41-44) = row order. */
void or_bucket_csr(int64_t N, int L, int64_t nb, const int32_t* bucket, int64_t* row_ptr, int32_t* idx) {
    for (int l = 0; l < L; l++) {
        int64_t* rp = row_ptr + (size_t)l * (nb + 1);
        memset(rp, 0, sizeof(int64_t) * (nb + 1));
        for (int64_t n = 0; n < N; n++) rp[bucket[n * L + l] + 1]++;
        for (int64_t b = 0; b < nb; b++) rp[b + 1] += rp[b];
        int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * nb);
        memcpy(cur, rp, sizeof(int64_t) * nb);
        for (int64_t n = 0; n < N; n++) idx[(size_t)l * N + cur[bucket[n * L + l]]++] = (int32_t)n;
        free(cur);
    }
}

static int cmp_i32(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    return (x > y) - (x < y);
}

/* get_LSH_[filtered_]combined_buckets (lsh_cube.hpp:77-106) with
 * getFilteredBucketFor (cust_hashtable.hpp:73-103): std::set<CustVector*>
 * orders by address = row index (one contiguous std::vector). */
int64_t or_lsh_query(int64_t N, int L, int k, int64_t nb, const int32_t* tuples, const int64_t* row_ptr,
                     const int32_t* idx, const int32_t* q_tuple, const int32_t* q_bucket,
                     int32_t* out, int64_t cap) {
    int64_t total = 0;
    for (int l = 0; l < L; l++) {
        const int64_t* rp = row_ptr + (size_t)l * (nb + 1);
        total += rp[q_bucket[l] + 1] - rp[q_bucket[l]];
    }
    int32_t* tmp = (int32_t*)malloc(sizeof(int32_t) * (total > 0 ? total : 1));
    int64_t m = 0;
    for (int l = 0; l < L; l++) {
        const int64_t* rp = row_ptr + (size_t)l * (nb + 1);
        for (int64_t p = rp[q_bucket[l]]; p < rp[q_bucket[l] + 1]; p++) {
            int32_t mem = idx[(size_t)l * N + p];
            int keep = 1;
            if (tuples && q_tuple)
                for (int i = 0; i < k; i++)
                    if (tuples[((size_t)mem * L + l) * k + i] != q_tuple[l * k + i]) { keep = 0; break; }
            if (keep) tmp[m++] = mem;
        }
    }
    qsort(tmp, m, sizeof(int32_t), cmp_i32);
    int64_t u = 0;
    for (int64_t i = 0; i < m; i++)
        if (i == 0 || tmp[i] != tmp[i - 1]) { if (u < cap) out[u] = tmp[i]; u++; }
    free(tmp);
    return u;
}

/* ----------------------------------------------------------------- hypercube */
void or_cube_h(int64_t N, int d, int k, const double* X, const float* V, const float* t, float w, int32_t* h) {
#pragma omp parallel for schedule(static)
    for (int64_t n = 0; n < N; n++)
        for (int i = 0; i < k; i++) h[n * k + i] = or_euclid_h(V + (size_t)i * d, X + n * d, d, t[i], w);
}

/* EuclideanFGen::generate (euclidean_f_gen.hpp:65-79) under HypercubeGen
 * (hypercube_gen.hpp:63-73): coin c~U_int{1,2} drawn from the shared engine on
 * first sight of h for f_i, bit = mod(h, c); vertex packs f_0 as MSB. */
int64_t or_cube_coins(int64_t N, int k, const int32_t* h, int32_t hmin, int32_t hspan,
                      int32_t* memo, uint32_t* state, int32_t* vertex) {
    int64_t draws = 0;
    for (int64_t n = 0; n < N; n++) {
        int v = 0;
        for (int i = 0; i < k; i++) {
            int32_t hv = h[n * k + i];
            int64_t off = (int64_t)hv - hmin;
            if (off < 0 || off >= hspan) return -1;
            int32_t* m = memo + (size_t)i * hspan + off;
            if (*m < 0) {
                int c = or_uniform_int(state, 1, 2);
                *m = (hv % c + c) % c;
                draws++;
            }
            v = (v << 1) + *m;
        }
        if (vertex) vertex[n] = v;
    }
    return draws;
}

void or_cube_cosine(int64_t N, int d, int k, const double* X, const double* R, int32_t* vertex) {
#pragma omp parallel for schedule(static)
    for (int64_t n = 0; n < N; n++) {
        int v = 0;
        for (int i = 0; i < k; i++) v = (v << 1) + or_cosine_h(R + (size_t)i * d, X + n * d, d);
        vertex[n] = v;
    }
}

/* get_hypercube_combined_buckets (lsh_cube.hpp:139-177) probe order with
 * get_num_hamming_dist_from (utils.cpp:22-50): main bucket, then Hamming
 * distance 1 (bit 0 .. k-1), distance 2 in lexicographic (i<j), ...; when
 * probes == 1 the distance-1 list is never built (:148-150). */
int64_t or_cube_probe_seq(int32_t vertex, int probes, int k, int32_t* out, int64_t cap) {
    int64_t n = 0;
    if (cap > 0) out[0] = vertex;
    n = 1;
    int remaining = probes;
    int dist = probes > 1 ? 1 : 2;
    int comb[64];
    while (remaining > 0 && dist <= k) {
        for (int i = 0; i < dist; i++) comb[i] = i;
        for (;;) {
            int m = 0;
            for (int i = 0; i < dist; i++) m |= 1 << comb[i];
            if (n < cap) out[n] = vertex ^ m;
            n++;
            if (--remaining == 0) break;
            int p = dist - 1;
            while (p >= 0 && comb[p] == k - dist + p) p--;
            if (p < 0) break;
            comb[p]++;
            for (int q = p + 1; q < dist; q++) comb[q] = comb[q - 1] + 1;
        }
        dist++;
    }
    return n;
}

/* -------------------------------------------------------------------- Lloyd */

/* CustVector::euclideanDistance (cust_vector.hpp:124-136), this = x, in = c. */
double or_euclid_dist(const double* x, const double* c, int d) {
    double acc = 0;
    for (int j = 0; j < d; j++) acc = acc + pow((double)x[j] - c[j], 2);
    return sqrt(acc);
}

/* CustVector::cosineDistance (cust_vector.hpp:139-155), this = x, in = c. */
static double cosine_dist(const double* x, const double* c, int d) {
    long double ip = 0.0L;
    for (int j = 0; j < d; j++) ip = ip + (long double)((double)x[j] * c[j]);
    double a = 0, b = 0;
    for (int j = 0; j < d; j++) { a = a + pow((double)x[j], 2); b = b + pow(c[j], 2); }
    double denom = sqrt(a) * sqrt(b);
    return 1 - (double)(ip / (long double)denom);
}

/* lloyds_assignment (assignment.hpp:54-80): strict '<' with the -1 sentinel,
 * then the centroid override (:77-78). */
void or_lloyd_assign(int64_t N, int d, int K, const double* X, const double* C, int metric,
                     const int32_t* src_rows, int32_t* assign, double* dist) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t n = 0; n < N; n++) {
        double mn = -1; int arg = 0;
        for (int c = 0; c < K; c++) {
            double dd = metric == 0 ? or_euclid_dist(X + n * d, C + (size_t)c * d, d)
                                    : cosine_dist(X + n * d, C + (size_t)c * d, d);
            if (mn == -1 || dd < mn) { mn = dd; arg = c; }
        }
        assign[n] = arg; dist[n] = mn;
    }
    if (src_rows)
        for (int c = 0; c < K; c++)
            if (src_rows[c] >= 0 && src_rows[c] < N) { assign[src_rows[c]] = c; dist[src_rows[c]] = 0; }   /* as lshkm_lloyd_assign: rows outside [0, N) ignored */
}

static double euclid_f64(const double* a, const double* b, int d) {
    double acc = 0;
    for (int j = 0; j < d; j++) acc = acc + pow(a[j] - b[j], 2);
    return sqrt(acc);
}

static double cosine_f64(const double* a, const double* b, int d) {
    long double ip = 0.0L;
    for (int j = 0; j < d; j++) ip = ip + (long double)(a[j] * b[j]);
    double x = 0, y = 0;
    for (int j = 0; j < d; j++) { x = x + pow(a[j], 2); y = y + pow(b[j], 2); }
    double denom = sqrt(x) * sqrt(y);
    return 1 - (double)(ip / (long double)denom);
}

/* k_means (update.hpp:37-86): per-cluster sequential fp64 sum in input order,
 * divide unless empty, continue iff some center moved > min_dist. */
int or_kmeans_update(int64_t N, int d, int K, const double* X, const int32_t* assign,
                     const double* C_old, int metric, double min_dist, double* C_new, int64_t* counts) {
    memset(C_new, 0, sizeof(double) * (size_t)K * d);
    memset(counts, 0, sizeof(int64_t) * K);
    for (int64_t n = 0; n < N; n++) {
        int a = assign[n];
        counts[a]++;
        double* c = C_new + (size_t)a * d;
        for (int j = 0; j < d; j++) c[j] = c[j] + (double)X[n * d + j];
    }
    for (int c = 0; c < K; c++)
        if ((double)counts[c] != 0)
            for (int j = 0; j < d; j++) C_new[(size_t)c * d + j] = C_new[(size_t)c * d + j] / (double)counts[c];
    for (int c = 0; c < K; c++) {
        double dd = metric == 0 ? euclid_f64(C_new + (size_t)c * d, C_old + (size_t)c * d, d)
                                : cosine_f64(C_new + (size_t)c * d, C_old + (size_t)c * d, d);
        if (dd > min_dist) return 1;
    }
    return 0;
}

/* ------------------------------------------------------------ initialization */

/* rand_selection (initialization.hpp:39-69): uniform rows, redrawn (and all
 * earlier picks re-checked) on a repeat. IDs are unique, so ID equality is
 * row equality. */
void or_rand_selection(uint64_t seed, int64_t N, int K, int32_t* rows) {
    uint32_t s = or_minstd_seed(seed);
    rows[0] = or_uniform_int(&s, 0, (int)(N - 1));
    for (int i = 1; i < K; i++) {
        int r = or_uniform_int(&s, 0, (int)(N - 1)), c = 0;
        while (c < i) {
            if (rows[c] == r) { r = or_uniform_int(&s, 0, (int)(N - 1)); c = 0; }
            else c++;
        }
        rows[i] = r;
    }
}

/* k_means_pp (initialization.hpp:71-156), row by row as the reference: min
 * over centroids 0..i-1 with the -1 sentinel and strict '<' (the ID-keyed
 * cache only memoises), max with strict '>' from 0, (min/max)^2 prefix-summed
 * in row order, uniform_real<double>(0, total) = canon * (total - 0) + 0, and
 * the custom binary search (:134-149). */
void or_kmeans_pp(int64_t N, int d, int K, const double* X, int metric, uint64_t seed, int32_t* rows) {
    uint32_t s = or_minstd_seed(seed);
    double* md = (double*)malloc(sizeof(double) * (size_t)N);
    double* cs = (double*)malloc(sizeof(double) * (size_t)K * d);
    rows[0] = or_uniform_int(&s, 0, (int)(N - 1));
    for (int i = 1; i < K; i++) {
        for (int j = 0; j < d; j++) cs[(size_t)(i - 1) * d + j] = (double)X[(size_t)rows[i - 1] * d + j];
        double mx = 0;
#pragma omp parallel for schedule(static)
        for (int64_t n = 0; n < N; n++) {
            double mn = -1;
            for (int c = 0; c < i; c++) {
                const double dd = metric == 0 ? or_euclid_dist(X + n * d, cs + (size_t)c * d, d)
                                              : cosine_dist(X + n * d, cs + (size_t)c * d, d);
                if (mn == -1 || dd < mn) mn = dd;
            }
            md[n] = mn;
        }
        for (int64_t n = 0; n < N; n++)
            if (md[n] > mx) mx = md[n];
        md[0] = md[0] / mx;
        md[0] = md[0] * md[0];
        for (int64_t n = 1; n < N; n++) {
            md[n] = md[n] / mx;
            md[n] = md[n] * md[n];
            md[n] = md[n] + md[n - 1];
        }
        const double rd = canon_d(&s) * (md[N - 1] - 0.0) + 0.0;
        int64_t left = 0, right = N - 1, pick = 0;
        if (rd > md[left]) {
            while (right - left > 1) {
                const int64_t m = left + (right - left) / 2;
                if (rd <= md[m]) right = m;
                else left = m;
            }
            pick = right;
        }
        rows[i] = (int32_t)pick;
    }
    free(md);
    free(cs);
}

/* ------------------------------------------------------------ recommendation */

/* CustVector::cosineSimilarity (cust_vector.hpp:158-174), this = a, in = b. */
static double cos_sim_f64(const double* a, const double* b, int d) {
    long double ip = 0.0L;
    for (int j = 0; j < d; j++) ip = ip + (long double)(a[j] * b[j]);
    double x = 0, y = 0;
    for (int j = 0; j < d; j++) { x = x + pow(a[j], 2); y = y + pow(b[j], 2); }
    double denom = sqrt(x) * sqrt(y);
    return (double)(ip / (long double)denom);
}

/* parallel_quickSort / parralel_partition (crypto_rec.hpp:234-277): Lomuto,
 * pivot = last, elements >= pivot to the front, recursion left then right. */
static void lomuto_desc(double* key, int32_t* val, int low, int high) {
    if (low < high) {
        const double pivot = key[high];
        int i = low - 1;
        for (int j = low; j <= high - 1; j++) {
            if (key[j] >= pivot) {
                i++;
                double tk = key[i]; key[i] = key[j]; key[j] = tk;
                int32_t tv = val[i]; val[i] = val[j]; val[j] = tv;
            }
        }
        double tk = key[i + 1]; key[i + 1] = key[high]; key[high] = tk;
        int32_t tv = val[i + 1]; val[i + 1] = val[high]; val[high] = tv;
        lomuto_desc(key, val, low, i);
        lomuto_desc(key, val, i + 2, high);
    }
}

/* get_P_closest (crypto_rec.hpp:213-231) per user q over its candidates
 * cand_idx[cand_ptr[q] .. cand_ptr[q+1]): similarities, the quicksort, first P.
 * out_idx / out_sim [nq][P]; out_cnt[q] = min(P, n). */
void or_p_closest(int d, const double* X, int64_t nq, const double* U, const int64_t* cand_ptr,
                  const int32_t* cand_idx, int P, int32_t* out_idx, double* out_sim, int32_t* out_cnt) {
    for (int64_t q = 0; q < nq; q++) {
        const int64_t o = cand_ptr[q];
        const int n = (int)(cand_ptr[q + 1] - o);
        double* s = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
        int32_t* r = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
        for (int i = 0; i < n; i++) {
            r[i] = cand_idx[o + i];
            s[i] = cos_sim_f64(X + (size_t)r[i] * d, U + (size_t)q * d, d);
        }
        lomuto_desc(s, r, 0, n - 1);
        const int c = n < P ? n : P;
        for (int i = 0; i < c; i++) { out_idx[q * P + i] = r[i]; out_sim[q * P + i] = s[i]; }
        out_cnt[q] = c;
        free(s); free(r);
    }
}

/* get_top_N_recom (crypto_rec.hpp:305-325) with get_predicted_user_sim
 * (:280-302) over the P-closest lists; unknown indexes per user as CSR
 * (ascending, std::set order); out [nq][N], padded with 0 (vector::resize). */
void or_top_n_recom(int d, const double* X, const double* x_mean, int64_t nq, const double* U,
                    const double* u_mean, const int64_t* unk_ptr, const int32_t* unk_idx, const int32_t* nb_idx,
                    const double* nb_sim, const int32_t* nb_cnt, int P, int N, int32_t* out) {
    for (int64_t q = 0; q < nq; q++) {
        const int64_t o = unk_ptr[q];
        const int m = (int)(unk_ptr[q + 1] - o);
        double* pred = (double*)malloc(sizeof(double) * (size_t)(m > 0 ? m : 1));
        int32_t* ix = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m > 0 ? m : 1));
        for (int u = 0; u < m; u++) {
            const int index = unk_idx[o + u];
            double main_sum = 0, abs_sum = 0;
            for (int i = 0; i < nb_cnt[q]; i++) {
                const double cs = nb_sim[q * P + i];
                abs_sum = abs_sum + fabs(cs);
                const int32_t r = nb_idx[q * P + i];
                main_sum = main_sum + (cs * (X[(size_t)r * d + index] - x_mean[r]));
            }
            double p = main_sum / abs_sum;
            p = p + u_mean[q];
            pred[u] = p;
            ix[u] = index;
        }
        lomuto_desc(pred, ix, 0, m - 1);
        for (int i = 0; i < N; i++) out[q * N + i] = i < m ? ix[i] : 0;
        free(pred); free(ix);
    }
}

/* get_top_N_recom(neighbors, user, N) -- the 3-argument overload
 * (crypto_rec.hpp:327-345) -- as the clustering recommenders call it
 * (main.cpp:260-269 with the user's own cluster, :353-373 with the cluster of
 * the user's nearest centroid). User q's neighbours are the members of cluster
 * ucl[q], crows[crow[c] .. crow[c+1]) in member order (separate_clusters_from_input,
 * utils.hpp:150-158); similarities cosineSimilarity(member, user) in that order
 * (:330-332); get_predicted_user_sim over all of them (:280-306); the
 * quicksort of the unknown indexes' predictions (:341); first N, 0-padded
 * (:343). Users of an empty cluster are skipped by main.cpp (:262, :366): -1
 * in every slot. out [nq][N]. */
void or_cluster_top_n(int d, const double* X, const double* x_mean, const int64_t* crow, const int32_t* crows,
                      int64_t nq, const double* U, const double* u_mean, const int32_t* ucl,
                      const int64_t* unk_ptr, const int32_t* unk_idx, int N, int32_t* out) {
    /* users are independent: one per thread (the full C5 check runs 1,024 users
     * over 10M member rows) */
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t q = 0; q < nq; q++) {
        const int c = ucl[q];
        const int64_t b = crow[c];
        const int n = (int)(crow[c + 1] - b);
        if (n == 0) {
            for (int i = 0; i < N; i++) out[q * N + i] = -1;
            continue;
        }
        const double* u = U + (size_t)q * d;
        double* sim = (double*)malloc(sizeof(double) * (size_t)n);
        for (int i = 0; i < n; i++) sim[i] = cos_sim_f64(X + (size_t)crows[b + i] * d, u, d);
        const int64_t o = unk_ptr[q];
        const int m = (int)(unk_ptr[q + 1] - o);
        double* pred = (double*)malloc(sizeof(double) * (size_t)(m > 0 ? m : 1));
        int32_t* ix = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m > 0 ? m : 1));
        for (int e = 0; e < m; e++) {
            const int index = unk_idx[o + e];
            double main_sum = 0, abs_sum = 0;
            for (int i = 0; i < n; i++) {
                const double cs = sim[i];
                abs_sum = abs_sum + fabs(cs);
                const int32_t r = crows[b + i];
                main_sum = main_sum + (cs * (X[(size_t)r * d + index] - x_mean[r]));
            }
            double p = main_sum / abs_sum;
            p = p + u_mean[q];
            pred[e] = p;
            ix[e] = index;
        }
        lomuto_desc(pred, ix, 0, m - 1);
        for (int i = 0; i < N; i++) out[q * N + i] = i < m ? ix[i] : 0;
        free(sim); free(pred); free(ix);
    }
}

void or_synth(uint64_t seed, int64_t row0, int64_t rows, int d, float* out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < rows; i++)
        for (int j = 0; j < d; j++) out[i * d + j] = lshkm_synth_value(seed, (uint64_t)(row0 + i), (uint64_t)d, (uint64_t)j);
}

void or_synth_normal(uint64_t seed, int64_t row0, int64_t rows, int d, float* out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < rows; i++)
        for (int j = 0; j < d; j++)
            out[i * d + j] = lshkm_synth_normal_value(seed, (uint64_t)(row0 + i), (uint64_t)d, (uint64_t)j);
}

/* ---------------------------------------------------------- range assignment */

/* find_min_vector_distance (utils.hpp:161-178) over the centroid rows: pairs
 * (i, j > i) in order, the -1 sentinel and strict '<'. */
static double min_pair_dist(int K, int d, const double* C, int metric) {
    double mn = -1;
    for (int i = 0; i < K; i++)
        for (int j = i + 1; j < K; j++) {
            const double dd = metric == 0 ? euclid_f64(C + (size_t)i * d, C + (size_t)j * d, d)
                                          : cosine_f64(C + (size_t)i * d, C + (size_t)j * d, d);
            if (mn == -1 || dd < mn) mn = dd;
        }
    return mn;
}

/* The reference's distanceMap (assignment.hpp:157,176-186), keyed by
 * (centroid key, row): open addressing over 64-bit keys. */
typedef struct { uint64_t* k; double* v; size_t cap; } dmap_t;
static size_t dmap_slot(const dmap_t* m, uint64_t key) {
    size_t h = (size_t)(lshkm_splitmix64(key) & (m->cap - 1));
    while (m->k[h] != ~0ull && m->k[h] != key) h = (h + 1) & (m->cap - 1);
    return h;
}

/* range_assignment (assignment.hpp:148-217) over the given combined buckets
 * (comb_ptr/comb_idx: centroid i's bucket rows in the reference's order),
 * preceded by remove_clustering and followed by lloyds_for_remaining
 * (:83-104) and the centroid override (:125-127, :143-145), as
 * lsh_range_assignment / cube_range_assignment (:108-145) run them.
 * key[K] (or NULL = all distinct): centroids with equal keys share distance
 * cache entries, as centroids with equal IDs do in the reference (e.g. every
 * "k_means_center" after k_means, update.hpp:46). Returns the passes of the
 * do-while loop. */
int or_range_assign(int64_t N, int d, int K, const double* X, const double* C, int metric,
                    const int64_t* comb_ptr, const int32_t* comb_idx, const int32_t* key,
                    const int32_t* src_rows, int32_t* assign, double* dist) {
    for (int64_t n = 0; n < N; n++) { assign[n] = -1; dist[n] = 0; }
    double radius = min_pair_dist(K, d, C, metric) / 2;
    double min_radius = 0;
    const int64_t total = comb_ptr[K];
    dmap_t m;
    m.cap = 16;
    while (m.cap < (size_t)(2 * total + 16)) m.cap <<= 1;
    m.k = (uint64_t*)malloc(m.cap * sizeof(uint64_t));
    m.v = (double*)malloc(m.cap * sizeof(double));
    for (size_t i = 0; i < m.cap; i++) m.k[i] = ~0ull;
    int passes = 0;
    int64_t assigned;
    do {
        assigned = 0;
        passes++;
        for (int i = 0; i < K; i++) {
            const uint64_t kc = (uint64_t)(uint32_t)(key ? key[i] : i) << 32;
            for (int64_t e = comb_ptr[i]; e < comb_ptr[i + 1]; e++) {
                const int32_t v = comb_idx[e];
                if (assign[v] == -1 || (assign[v] != -1 && dist[v] >= min_radius)) {
                    const size_t h = dmap_slot(&m, kc | (uint32_t)v);
                    double dd;
                    if (m.k[h] != ~0ull) dd = m.v[h];
                    else {
                        dd = metric == 0 ? or_euclid_dist(X + (size_t)v * d, C + (size_t)i * d, d)
                                         : cosine_dist(X + (size_t)v * d, C + (size_t)i * d, d);
                        m.k[h] = kc | (uint32_t)v;
                        m.v[h] = dd;
                    }
                    if (dd >= min_radius && dd < radius) {
                        if (assign[v] == -1) { assign[v] = i; dist[v] = dd; assigned++; }
                        else if (dist[v] > dd) { assign[v] = i; dist[v] = dd; assigned++; }
                    }
                }
            }
            min_radius = radius;
            radius = radius * 2;
        }
    } while (assigned > 0);
    free(m.k); free(m.v);
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t n = 0; n < N; n++) {
        if (assign[n] != -1) continue;
        double mn = -1; int arg = 0;
        for (int c = 0; c < K; c++) {
            double dd = metric == 0 ? or_euclid_dist(X + n * d, C + (size_t)c * d, d)
                                    : cosine_dist(X + n * d, C + (size_t)c * d, d);
            if (mn == -1 || dd < mn) { mn = dd; arg = c; }
        }
        assign[n] = arg; dist[n] = mn;
    }
    if (src_rows)
        for (int c = 0; c < K; c++)
            if (src_rows[c] >= 0 && src_rows[c] < N) { assign[src_rows[c]] = c; dist[src_rows[c]] = 0; }   /* as lshkm_lloyd_assign: rows outside [0, N) ignored */
    return passes;
}

/* ---------------------------------------------------------------- silhouette */

/* silhouette_cluster (silhouette.hpp:31-80) over separate_clusters_from_input
 * (utils.hpp:150-158), silhouette_of_i (:83-144). The reference's distance
 * cache is left out: it returns d(x_j, x_i) for d(x_i, x_j), which is the same
 * double in both metrics (unique IDs). out[K+1]; s[N] (may be NULL) per row. */
void or_silhouette(int64_t N, int d, int K, const double* X, const int32_t* assign, const double* C, int metric,
                   double* out, double* s) {
    int32_t* near = (int32_t*)malloc(sizeof(int32_t) * (size_t)K);
    for (int c = 0; c < K; c++) {
        double mn = -1; int arg = 0;
        for (int i = 0; i < K; i++) {
            if (i == c) continue;
            const double dd = metric == 0 ? euclid_f64(C + (size_t)c * d, C + (size_t)i * d, d)
                                          : cosine_f64(C + (size_t)c * d, C + (size_t)i * d, d);
            if (mn == -1 || dd < mn) { mn = dd; arg = i; }
        }
        near[c] = arg;
    }
    int64_t* cnt = (int64_t*)calloc((size_t)K + 1, sizeof(int64_t));
    for (int64_t n = 0; n < N; n++) cnt[assign[n] + 1]++;
    for (int c = 0; c < K; c++) cnt[c + 1] += cnt[c];
    int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)K);
    int32_t* rows = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
    for (int c = 0; c < K; c++) fill[c] = cnt[c];
    for (int64_t n = 0; n < N; n++) rows[fill[assign[n]]++] = (int32_t)n;
    double* sv = (double*)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1));
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t p = 0; p < N; p++) {
        const int32_t r = rows[p];
        const int c = assign[r];
        double* xr = (double*)malloc(sizeof(double) * (size_t)d);
        double a = 0, b = 0;
        for (int64_t j = cnt[c]; j < cnt[c + 1]; j++) {
            for (int t = 0; t < d; t++) xr[t] = X[(size_t)rows[j] * d + t];
            a = a + (metric == 0 ? or_euclid_dist(X + (size_t)r * d, xr, d)
                                 : cosine_dist(X + (size_t)r * d, xr, d));
        }
        if (cnt[c + 1] - cnt[c] != 1) a = a / (double)(size_t)(cnt[c + 1] - cnt[c] - 1);
        const int nc = near[c];
        for (int64_t j = cnt[nc]; j < cnt[nc + 1]; j++) {
            for (int t = 0; t < d; t++) xr[t] = X[(size_t)rows[j] * d + t];
            b = b + (metric == 0 ? or_euclid_dist(X + (size_t)r * d, xr, d)
                                 : cosine_dist(X + (size_t)r * d, xr, d));
        }
        b = b / (double)(size_t)(cnt[nc + 1] - cnt[nc]);
        double mx = a;
        if (b > a) mx = b;
        sv[p] = (b - a) / mx;
        if (s) s[r] = sv[p];
        free(xr);
    }
    out[K] = 0;
    for (int c = 0; c < K; c++) {
        out[c] = 0;
        for (int64_t p = cnt[c]; p < cnt[c + 1]; p++) out[c] = out[c] + sv[p];
        out[K] = out[K] + out[c];
        out[c] = out[c] / (double)(size_t)(cnt[c + 1] - cnt[c]);
    }
    out[K] = out[K] / (double)(int)N;
    free(near); free(cnt); free(fill); free(rows); free(sv);
}
