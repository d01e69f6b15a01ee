/*
 * lshkm_compat.hpp — C++ drop-in for the reference's header-template interface
 * of the hot path, on top of the C ABI in lshkm.h.
 *
 * Include it AFTER the reference's own headers (it uses their CustVector,
 * CustHashtable and HashGenerator types and adds none of its own):
 *
 *     #include "lsh_cube.hpp"                      // lib/lsh_cube.hpp
 *     #include "clustering_phases/assignment.hpp"
 *     #include "clustering_phases/update.hpp"
 *     #include "lshkm_compat.hpp"                  // this file; link -llshkm
 *
 * and call lshkm_compat::X where the reference calls X:
 *
 *   create_LSH_hashtables   lib/lsh_cube.hpp:44-74
 *   create_hypercube        lib/lsh_cube.hpp:108-136
 *   lloyds_assignment       lib/clustering_phases/assignment.hpp:54-80
 *   k_means                 lib/clustering_phases/update.hpp:37-86
 *   k_means_pp              lib/clustering_phases/initialization.hpp:71-156
 *   rand_selection          lib/clustering_phases/initialization.hpp:39-69
 *   get_P_closest           lib/crypto_rec.hpp:213-231
 *   get_top_N_recom (both overloads)  lib/crypto_rec.hpp:309-345
 *
 * Same signatures, same return values and the same ownership as the
 * reference: the hashtables are real CustHashtable objects (the caller deletes
 * them; each deletes its generator), so get_LSH_combined_buckets,
 * get_LSH_filtered_combined_buckets and get_hypercube_combined_buckets
 * (lsh_cube.hpp:77-177) and every CustHashtable method work on them
 * unchanged. Their generators are GPU-backed HashGenerator plugins
 * (hash_generator.hpp:19-31): the dataset rows are hashed in one device pass
 * at creation, a query vector in one device call shared by the L tables.
 * k_means allocates and deletes centers exactly as update.hpp:66-84 does.
 *
 * The seed: the reference seeds from system_clock (lsh_cube.hpp:48-51,
 * 112-114); the overloads without a seed do the same, the ones with a trailing
 * `seed` argument make a run reproducible.
 *
 * Data: vectors go to the device as fp32 rows when every component is an fp32
 * value (the tuned storage: the synthetic and proj-2 inputs are) and as fp64
 * rows otherwise (the `_f64` entry points: general doubles such as the
 * recommender's user vectors, crypto_rec.hpp:78-140); the results are the
 * same either way. Centroids are fp64. Dataset rows are hashed when the table
 * is built, as the reference's insertVector does; re-hashing a dataset row
 * later returns that hash (the reference never mutates its input vectors).
 *
 * Errors from the library throw lshkm_compat::Error (std::runtime_error). The
 * device is ordinal LSHKM_DEVICE (environment, default 0); one context per
 * thread.
 */
#ifndef LSHKM_COMPAT_HPP
#define LSHKM_COMPAT_HPP

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "lshkm.h"

namespace lshkm_compat {

struct Error : std::runtime_error {
    explicit Error(const std::string& m) : std::runtime_error("liblshkm: " + m) {}
};

inline void check(int rc) {
    if (rc != LSHKM_OK) throw Error(lshkm_last_error());
}

// ------------------------------------------------------------ context / memory
// The shim is a zero-change drop-in for the reference's semantics, so its
// contexts run in LSHKM_DIST_EXACT mode: every distance a CustVector receives
// (setCluster, assignment.hpp:73-76) is the reference's fp64 chain.
// set_distance_mode(LSHKM_DIST_CERTIFIED) opts the calling thread into the
// faster certified distances (<= 2^-20 relative; cluster IDs unchanged).
class Context {
public:
    Context() {
        const char* env = std::getenv("LSHKM_DEVICE");
        check(lshkm_ctx_create(env ? std::atoi(env) : 0, &h_));
        check(lshkm_ctx_set_dist_mode(h_, LSHKM_DIST_EXACT));
    }
    ~Context() { lshkm_ctx_destroy(h_); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    lshkm_ctx get() const { return h_; }

private:
    lshkm_ctx h_ = nullptr;
};

inline lshkm_ctx context() {
    static thread_local Context c;
    return c.get();
}

// LSHKM_DIST_EXACT (the shim's default) or LSHKM_DIST_CERTIFIED for the
// calling thread's context.
inline void set_distance_mode(int mode) { check(lshkm_ctx_set_dist_mode(context(), mode)); }

// Device allocation owned by the calling thread's context.
class DevMem {
public:
    DevMem() = default;
    explicit DevMem(size_t bytes) { check(lshkm_dev_alloc(context(), (int64_t)bytes, &p_)); }
    ~DevMem() { if (p_) lshkm_dev_free(context(), p_); }
    DevMem(DevMem&& o) noexcept : p_(o.p_) { o.p_ = nullptr; }
    DevMem& operator=(DevMem&& o) noexcept { std::swap(p_, o.p_); return *this; }
    DevMem(const DevMem&) = delete;
    DevMem& operator=(const DevMem&) = delete;
    template <typename U> U* as() const { return static_cast<U*>(p_); }

private:
    void* p_ = nullptr;
};

template <typename U>
DevMem upload(const U* host, size_t n) {
    DevMem m(n * sizeof(U));
    check(lshkm_memcpy_h2d(context(), m.as<void>(), host, (int64_t)(n * sizeof(U))));
    return m;
}

template <typename U>
void download(U* host, const DevMem& m, size_t n) {
    check(lshkm_memcpy_d2h(context(), host, m.as<void>(), (int64_t)(n * sizeof(U))));
}

inline int metric_of(const std::string& metric) {
    if (metric == "euclidean") return LSHKM_METRIC_EUCLIDEAN;
    if (metric == "cosine") return LSHKM_METRIC_COSINE;
    throw std::invalid_argument("lshkm_compat: unknown metric '" + metric + "'");
}

inline unsigned long clock_seed() {   // lsh_cube.hpp:48
    return std::chrono::system_clock::now().time_since_epoch().count();
}

// Rows on the device: fp32 when every component is an fp32 value, else fp64.
struct DevRows {
    DevMem m;
    bool f64 = false;
    const float* f() const { return m.as<float>(); }
    const double* d() const { return m.as<double>(); }
};

template <typename T>
const std::vector<T>& dims_of(CustVector<T>& v, size_t d) {
    const std::vector<T>& x = *v.getDimensions();
    if (x.size() != d)
        throw std::invalid_argument("lshkm_compat: vector '" + v.getId() + "' has " + std::to_string(x.size()) +
                                    " dimensions, expected " + std::to_string(d));
    return x;
}

template <typename T>
DevRows upload_rows(CustVector<T>* const* vs, size_t n, size_t d) {
    bool fp32 = true;
    for (size_t i = 0; i < n && fp32; i++) {
        const std::vector<T>& x = dims_of(*vs[i], d);
        for (size_t j = 0; j < d; j++)
            if (static_cast<T>(static_cast<float>(x[j])) != x[j]) { fp32 = false; break; }
    }
    DevRows r;
    r.f64 = !fp32;
    if (fp32) {
        std::vector<float> X(n * d);
        for (size_t i = 0; i < n; i++)
            for (size_t j = 0; j < d; j++) X[i * d + j] = static_cast<float>((*vs[i]->getDimensions())[j]);
        r.m = upload(X.data(), X.size());
    } else {
        std::vector<double> X(n * d);
        for (size_t i = 0; i < n; i++)
            for (size_t j = 0; j < d; j++) X[i * d + j] = static_cast<double>((*vs[i]->getDimensions())[j]);
        r.m = upload(X.data(), X.size());
    }
    return r;
}

template <typename T>
DevRows upload_rows(std::vector<CustVector<T>>& vs, size_t d) {
    std::vector<CustVector<T>*> p(vs.size());
    for (size_t i = 0; i < vs.size(); i++) p[i] = &vs[i];
    return upload_rows(p.data(), p.size(), d);
}

template <typename T>
DevRows upload_row(CustVector<T>& v, size_t d) {
    CustVector<T>* p = &v;
    return upload_rows(&p, 1, d);
}

// Index of `v` in the dataset [base, base + n), or -1.
template <typename T>
int64_t row_of(const CustVector<T>* v, const CustVector<T>* base, int64_t n) {
    if (!base || v < base || v >= base + n) return -1;
    return v - base;
}

// ---------------------------------------------------------------- LSH tables
// State shared by the L generators of one create_LSH_hashtables call.
template <typename T>
struct LshState {
    lshkm_lsh h = nullptr;
    int metric = 0, k = 0, L = 0;
    size_t d = 0;
    const CustVector<T>* base = nullptr;
    int64_t N = 0;
    std::vector<int32_t> value;    // [N][L] phi (euclidean) or g (cosine)
    std::vector<int32_t> tuples;   // [N][L][k] h tuples (euclidean)
    // last query, hashed once for all L tables
    const CustVector<T>* q_ptr = nullptr;
    std::vector<T> q_dims;
    std::vector<int32_t> q_value, q_tuples;

    ~LshState() { lshkm_lsh_destroy(h); }

    void hash_query(CustVector<T>* v) {
        if (v == q_ptr && *v->getDimensions() == q_dims) return;
        const DevRows X = upload_row(*v, d);
        DevMem val(sizeof(int32_t) * L), tup(sizeof(int32_t) * L * k);
        const bool eu = metric == LSHKM_METRIC_EUCLIDEAN;
        int32_t* tp = eu ? tup.as<int32_t>() : nullptr;
        check(X.f64 ? lshkm_lsh_hash_f64(h, X.d(), 1, tp, val.as<int32_t>(), nullptr)
                    : lshkm_lsh_hash(h, X.f(), 1, tp, val.as<int32_t>(), nullptr));
        q_value.resize(L);
        download(q_value.data(), val, L);
        q_tuples.assign(eu ? (size_t)L * k : 0, 0);
        if (eu) download(q_tuples.data(), tup, (size_t)L * k);
        q_ptr = v;
        q_dims = *v->getDimensions();
    }
};

// EuclideanPhiGen (euclidean_phi_gen.hpp:77-92) / CosineGGen
// (cosine_g_gen.hpp:56-66) of table `l`, answered by the device.
template <typename T>
class GpuLshGenerator : public HashGenerator<T> {
public:
    GpuLshGenerator(std::shared_ptr<LshState<T>> st, int table) : st_(std::move(st)), l_(table) {}

    int generate(CustVector<T>* v) override {
        const LshState<T>& s = *st_;
        const int64_t r = row_of<T>(v, s.base, s.N);
        const int32_t* tup;
        int value;
        if (r >= 0) {
            value = s.value[(size_t)r * s.L + l_];
            tup = s.tuples.empty() ? nullptr : &s.tuples[((size_t)r * s.L + l_) * s.k];
        } else {
            st_->hash_query(v);
            value = s.q_value[l_];
            tup = s.q_tuples.empty() ? nullptr : &s.q_tuples[(size_t)l_ * s.k];
        }
        // first write wins per ID, as id_to_det_hashes.emplace (euclidean_phi_gen.hpp:94)
        if (tup) detailed_.emplace(v->getId(), std::vector<int>(tup, tup + s.k));
        return value;
    }
    bool hasDetailedHash() override { return st_->metric == LSHKM_METRIC_EUCLIDEAN; }
    std::unordered_map<std::string, std::vector<int>>* getDetailedHashes() override { return &detailed_; }
    unsigned long getSize() override {
        unsigned long size = sizeof(*this);
        for (const auto& e : detailed_) size += e.first.capacity() + e.second.capacity() * sizeof(int) + 64;
        return size;
    }

private:
    std::shared_ptr<LshState<T>> st_;
    int l_;
    std::unordered_map<std::string, std::vector<int>> detailed_;
};

template <typename T>
std::vector<CustHashtable<T>*> create_LSH_hashtables(std::vector<CustVector<T>>& input_vectors,
                                                     const std::string metric_type, int k, int L,
                                                     int lsh_bucket_div, double euclidean_h_w, unsigned long seed) {
    if (input_vectors.empty() || k < 1 || L < 1) throw std::invalid_argument("lshkm_compat: empty input or k, L < 1");
    auto st = std::make_shared<LshState<T>>();
    st->metric = metric_of(metric_type);
    st->k = k;
    st->L = L;
    st->d = input_vectors[0].getDimensions()->size();
    st->base = input_vectors.data();
    st->N = (int64_t)input_vectors.size();
    const int d = (int)st->d;
    const bool eu = st->metric == LSHKM_METRIC_EUCLIDEAN;
    const float w = (float)euclidean_h_w;   // EuclideanHGen stores float (euclidean_h_gen.hpp:36)
    const int64_t nb = eu ? (int64_t)(input_vectors.size() / lsh_bucket_div) : (int64_t)1 << k;
    if (nb < 1) throw std::invalid_argument("lshkm_compat: N / lsh_bucket_div is 0 buckets");

    uint32_t state = 0;
    if (eu) {
        std::vector<float> V((size_t)L * k * d), t((size_t)L * k);
        std::vector<int32_t> r((size_t)L * k);
        check(lshkm_params_lsh_euclidean(seed, L, k, d, w, V.data(), t.data(), r.data(), &state));
        check(lshkm_lsh_create(context(), st->metric, d, k, L, nb, w, V.data(), t.data(), r.data(), nullptr, &st->h));
    } else {
        std::vector<double> R((size_t)L * k * d);
        check(lshkm_params_lsh_cosine(seed, L, k, d, R.data(), &state));
        check(lshkm_lsh_create(context(), st->metric, d, k, L, nb, w, nullptr, nullptr, nullptr, R.data(), &st->h));
    }

    // every row, every table in one device pass
    const size_t N = (size_t)st->N;
    const DevRows Xd = upload_rows(input_vectors, st->d);
    DevMem val(sizeof(int32_t) * N * L), tup(eu ? sizeof(int32_t) * N * L * k : 0);
    int32_t* tp = eu ? tup.as<int32_t>() : nullptr;
    check(Xd.f64 ? lshkm_lsh_hash_f64(st->h, Xd.d(), st->N, tp, val.as<int32_t>(), nullptr)
                 : lshkm_lsh_hash(st->h, Xd.f(), st->N, tp, val.as<int32_t>(), nullptr));
    st->value.resize(N * L);
    download(st->value.data(), val, N * L);
    if (eu) {
        st->tuples.resize(N * L * k);
        download(st->tuples.data(), tup, N * L * k);
    }

    // tables in the reference's order, rows inserted in row order (lsh_cube.hpp:53-71)
    std::vector<CustHashtable<T>*> tables;
    tables.reserve(L);
    for (int l = 0; l < L; l++) {
        tables.emplace_back(new CustHashtable<T>(new GpuLshGenerator<T>(st, l), (int)nb));
        for (size_t i = 0; i < N; i++) tables[l]->insertVector(&input_vectors[i]);
    }
    return tables;
}

template <typename T>
std::vector<CustHashtable<T>*> create_LSH_hashtables(std::vector<CustVector<T>>& input_vectors,
                                                     const std::string metric_type, int k, int L,
                                                     int lsh_bucket_div, double euclidean_h_w) {
    return create_LSH_hashtables(input_vectors, metric_type, k, L, lsh_bucket_div, euclidean_h_w, clock_seed());
}

// ----------------------------------------------------------------- hypercube
template <typename T>
struct CubeState {
    lshkm_cube h = nullptr;
    size_t d = 0;
    const CustVector<T>* base = nullptr;
    int64_t N = 0;
    std::vector<int32_t> vertex;   // [N]
    ~CubeState() { lshkm_cube_destroy(h); }
};

// HypercubeGen (hypercube_gen.hpp:63-73) over k EuclideanFGen / CosineHGen,
// answered by the device; a query's unseen h values draw their coins from the
// continued engine (euclidean_f_gen.hpp:65-79).
template <typename T>
class GpuCubeGenerator : public HashGenerator<T> {
public:
    explicit GpuCubeGenerator(std::shared_ptr<CubeState<T>> st) : st_(std::move(st)) {}

    int generate(CustVector<T>* v) override {
        const CubeState<T>& s = *st_;
        const int64_t r = row_of<T>(v, s.base, s.N);
        if (r >= 0) return s.vertex[(size_t)r];
        const DevRows X = upload_row(*v, s.d);
        DevMem vert(sizeof(int32_t));
        check(X.f64 ? lshkm_cube_vertices_f64(s.h, X.d(), 1, vert.as<int32_t>())
                    : lshkm_cube_vertices(s.h, X.f(), 1, vert.as<int32_t>()));
        int32_t out = 0;
        download(&out, vert, 1);
        return out;
    }
    bool hasDetailedHash() override { return false; }
    std::unordered_map<std::string, std::vector<int>>* getDetailedHashes() override { return nullptr; }
    unsigned long getSize() override { return sizeof(*this) + st_->vertex.capacity() * sizeof(int32_t); }

private:
    std::shared_ptr<CubeState<T>> st_;
};

template <typename T>
CustHashtable<T>* create_hypercube(std::vector<CustVector<T>>& input_vectors, const std::string metric_type, int k,
                                   double euclidean_h_w, unsigned long seed) {
    if (input_vectors.empty() || k < 1 || k > 30) throw std::invalid_argument("lshkm_compat: empty input or k out of range");
    auto st = std::make_shared<CubeState<T>>();
    const int metric = metric_of(metric_type);
    st->d = input_vectors[0].getDimensions()->size();
    st->base = input_vectors.data();
    st->N = (int64_t)input_vectors.size();
    const int d = (int)st->d;
    const float w = (float)euclidean_h_w;
    uint32_t state = 0;
    if (metric == LSHKM_METRIC_EUCLIDEAN) {
        std::vector<float> V((size_t)k * d), t(k);
        check(lshkm_params_cube_euclidean(seed, k, d, w, V.data(), t.data(), &state));
        check(lshkm_cube_create(context(), metric, d, k, w, V.data(), t.data(), nullptr, state, &st->h));
    } else {
        std::vector<double> R((size_t)k * d);
        check(lshkm_params_cube_cosine(seed, k, d, R.data(), &state));
        check(lshkm_cube_create(context(), metric, d, k, w, nullptr, nullptr, R.data(), state, &st->h));
    }
    // the build draws the coins in (row, f) order, as the insert loop (lsh_cube.hpp:132-133)
    const size_t N = (size_t)st->N;
    const DevRows Xd = upload_rows(input_vectors, st->d);
    check(Xd.f64 ? lshkm_cube_build_f64(st->h, Xd.d(), st->N) : lshkm_cube_build(st->h, Xd.f(), st->N));
    DevMem vert(sizeof(int32_t) * N);
    // all h seen: no draws
    check(Xd.f64 ? lshkm_cube_vertices_f64(st->h, Xd.d(), st->N, vert.as<int32_t>())
                 : lshkm_cube_vertices(st->h, Xd.f(), st->N, vert.as<int32_t>()));
    st->vertex.resize(N);
    download(st->vertex.data(), vert, N);

    CustHashtable<T>* cube = new CustHashtable<T>(new GpuCubeGenerator<T>(st), 1 << k);
    for (size_t i = 0; i < N; i++) cube->insertVector(&input_vectors[i]);
    return cube;
}

template <typename T>
CustHashtable<T>* create_hypercube(std::vector<CustVector<T>>& input_vectors, const std::string metric_type, int k,
                                   double euclidean_h_w) {
    return create_hypercube(input_vectors, metric_type, k, euclidean_h_w, clock_seed());
}

// ------------------------------------------------------------------- k-means
template <typename T>
std::vector<double> pack_centers(std::vector<CustVector<T>*>& centers, size_t d) {
    std::vector<double> C(centers.size() * d);
    for (size_t c = 0; c < centers.size(); c++) {
        const std::vector<T>& x = *centers[c]->getDimensions();
        if (x.size() != d) throw std::invalid_argument("lshkm_compat: center dimension mismatch");
        for (size_t j = 0; j < d; j++) C[c * d + j] = static_cast<double>(x[j]);
    }
    return C;
}

// lloyds_assignment (assignment.hpp:54-80): nearest centroid (strict '<',
// first index wins) and its distance for every vector, then each centroid
// assigned to its own cluster at distance 0.
template <typename T>
void lloyds_assignment(std::vector<CustVector<T>>& input_vectors, std::vector<CustVector<T>*>& centroids,
                       std::string metric_type) {
    const int metric = metric_of(metric_type);
    if (input_vectors.empty() || centroids.empty()) {
        for (size_t c = 0; c < centroids.size(); c++) centroids[c]->setCluster((int)c, 0);
        return;
    }
    const size_t N = input_vectors.size(), K = centroids.size(), d = input_vectors[0].getDimensions()->size();
    const DevRows Xd = upload_rows(input_vectors, d);
    std::vector<double> C = pack_centers(centroids, d);
    std::vector<int32_t> src(K);
    for (size_t c = 0; c < K; c++) src[c] = (int32_t)row_of<T>(centroids[c], input_vectors.data(), (int64_t)N);
    DevMem Cd = upload(C.data(), C.size());
    DevMem ad(sizeof(int32_t) * N), dd(sizeof(double) * N);
    check(Xd.f64 ? lshkm_lloyd_assign_f64(context(), Xd.d(), (int64_t)N, (int)d, Cd.as<double>(), (int)K, metric,
                                          src.data(), ad.as<int32_t>(), dd.as<double>())
                 : lshkm_lloyd_assign(context(), Xd.f(), (int64_t)N, (int)d, Cd.as<double>(), (int)K, metric,
                                      src.data(), ad.as<int32_t>(), dd.as<double>()));
    std::vector<int32_t> a(N);
    std::vector<double> dist(N);
    download(a.data(), ad, N);
    download(dist.data(), dd, N);
    for (size_t i = 0; i < N; i++) input_vectors[i].setCluster(a[i], dist[i]);
    // centroids outside the dataset too, in centroid order (assignment.hpp:77-78)
    for (size_t c = 0; c < K; c++) centroids[c]->setCluster((int)c, 0);
}

// k_means (update.hpp:37-86): per-cluster means of the members in row order;
// if some center moved more than min_dist, every center is replaced by a new
// "k_means_center" vector (old ones with that ID deleted) and true returned,
// else the centers are left alone and false returned.
template <typename T>
bool k_means(std::vector<CustVector<T>>& input_vectors, std::vector<CustVector<T>*>& centers, std::string metric_type,
             double min_dist) {
    // the reference accumulates in the vector type (cust_vector.hpp:179-184);
    // the device sums are fp64, i.e. the reference's CustVector<double> (main.cpp:86)
    static_assert(std::is_same<T, double>::value, "lshkm_compat::k_means matches CustVector<double> only");
    const int metric = metric_of(metric_type);
    if (centers.empty()) return false;
    const size_t N = input_vectors.size(), K = centers.size(), d = centers[0]->getDimensions()->size();
    const DevRows Xd = upload_rows(input_vectors, d);
    std::vector<int32_t> a(N);
    for (size_t i = 0; i < N; i++) {
        a[i] = input_vectors[i].getCluster();
        if (a[i] < 0 || (size_t)a[i] >= K)
            throw std::out_of_range("lshkm_compat: vector '" + input_vectors[i].getId() + "' has no cluster in [0, K)");
    }
    std::vector<double> C = pack_centers(centers, d);
    DevMem ad = upload(a.data(), N), Cd = upload(C.data(), C.size());
    DevMem Cn(sizeof(double) * K * d);
    int cont = 0;
    check(Xd.f64 ? lshkm_kmeans_update_f64(context(), Xd.d(), (int64_t)N, (int)d, ad.as<int32_t>(), Cd.as<double>(),
                                           (int)K, metric, min_dist, Cn.as<double>(), nullptr, &cont)
                 : lshkm_kmeans_update(context(), Xd.f(), (int64_t)N, (int)d, ad.as<int32_t>(), Cd.as<double>(),
                                       (int)K, metric, min_dist, Cn.as<double>(), nullptr, &cont));
    if (!cont) return false;
    std::vector<double> Cnew(K * d);
    download(Cnew.data(), Cn, K * d);
    for (size_t c = 0; c < K; c++) {
        std::vector<T> dims(d);
        for (size_t j = 0; j < d; j++) dims[j] = static_cast<T>(Cnew[c * d + j]);
        if (centers[c]->getId() == "k_means_center") delete centers[c];
        centers[c] = new CustVector<T>("k_means_center", dims);
    }
    return true;
}

// ------------------------------------------------------------ initialization
// k_means_pp (initialization.hpp:71-156): pointers to the chosen input vectors.
// Vector IDs must be unique (the reference's distance cache is keyed by them).
template <typename T>
std::vector<CustVector<T>*> k_means_pp(std::vector<CustVector<T>>& input_vectors, int cluster_num,
                                       std::string metric_type, unsigned long seed) {
    const int metric = metric_of(metric_type);
    if (input_vectors.empty() || cluster_num < 1) throw std::invalid_argument("lshkm_compat: empty input or K < 1");
    const size_t N = input_vectors.size(), d = input_vectors[0].getDimensions()->size();
    const DevRows Xd = upload_rows(input_vectors, d);
    std::vector<int32_t> rows(cluster_num);
    check(Xd.f64 ? lshkm_kmeans_pp_f64(context(), Xd.d(), (int64_t)N, (int)d, cluster_num, metric, seed, rows.data())
                 : lshkm_kmeans_pp(context(), Xd.f(), (int64_t)N, (int)d, cluster_num, metric, seed, rows.data()));
    std::vector<CustVector<T>*> centroids(cluster_num);
    for (int i = 0; i < cluster_num; i++) centroids[i] = &input_vectors[rows[i]];
    return centroids;
}

template <typename T>
std::vector<CustVector<T>*> k_means_pp(std::vector<CustVector<T>>& input_vectors, int cluster_num,
                                       std::string metric_type) {
    return k_means_pp(input_vectors, cluster_num, metric_type, clock_seed());
}

// rand_selection (initialization.hpp:39-69).
template <typename T>
std::vector<CustVector<T>*> rand_selection(std::vector<CustVector<T>>& input_vectors, int cluster_num,
                                           unsigned long seed) {
    std::vector<int32_t> rows(cluster_num > 0 ? cluster_num : 0);
    check(lshkm_rand_selection(seed, (int64_t)input_vectors.size(), cluster_num, rows.data()));
    std::vector<CustVector<T>*> centroids(cluster_num);
    for (int i = 0; i < cluster_num; i++) centroids[i] = &input_vectors[rows[i]];
    return centroids;
}

template <typename T>
std::vector<CustVector<T>*> rand_selection(std::vector<CustVector<T>>& input_vectors, int cluster_num) {
    return rand_selection(input_vectors, cluster_num, clock_seed());
}

// ------------------------------------------------------------ recommendation
// get_P_closest (crypto_rec.hpp:213-231): sorts `neighbors` by similarity to
// `user` as the reference's quicksort does, keeps the first P, returns their
// similarities. fp64 throughout (no fp32 restriction here).
template <typename T>
std::vector<double> get_P_closest(std::vector<CustVector<T>*>& neighbors, CustVector<T>& user, int P) {
    static_assert(std::is_same<T, double>::value, "lshkm_compat::get_P_closest matches CustVector<double> only");
    const size_t n = neighbors.size(), d = user.getDimensions()->size();
    if (n == 0 || P < 1) return std::vector<double>();
    std::vector<double> X(n * d);
    for (size_t i = 0; i < n; i++) {
        const std::vector<T>& x = *neighbors[i]->getDimensions();
        if (x.size() != d) throw std::invalid_argument("lshkm_compat: neighbour dimension mismatch");
        for (size_t j = 0; j < d; j++) X[i * d + j] = x[j];
    }
    std::vector<int64_t> ptr = {0, (int64_t)n};
    std::vector<int32_t> cand(n);
    for (size_t i = 0; i < n; i++) cand[i] = (int32_t)i;
    DevMem Xd = upload(X.data(), X.size()), Ud = upload(user.getDimensions()->data(), d);
    DevMem pd = upload(ptr.data(), 2), cd = upload(cand.data(), n);
    DevMem oi(sizeof(int32_t) * P), os(sizeof(double) * P), oc(sizeof(int32_t));
    check(lshkm_p_closest(context(), Xd.as<double>(), (int64_t)n, (int)d, Ud.as<double>(), 1, pd.as<int64_t>(),
                          cd.as<int32_t>(), P, oi.as<int32_t>(), os.as<double>(), oc.as<int32_t>()));
    int32_t c = 0;
    download(&c, oc, 1);
    std::vector<int32_t> idx(P);
    std::vector<double> sim(P);
    download(idx.data(), oi, P);
    download(sim.data(), os, P);
    // the reference sorts the whole vector, then resizes it to P if longer:
    // either way the caller sees the first min(n, P) in sorted order
    std::vector<CustVector<T>*> sorted(c);
    for (int i = 0; i < c; i++) sorted[i] = neighbors[idx[i]];
    neighbors = sorted;
    sim.resize(c);
    return sim;
}

// get_top_N_recom (crypto_rec.hpp:305-325) with the similarities of get_P_closest.
template <typename T>
std::vector<int> get_top_N_recom(std::vector<CustVector<T>*>& neighbors, CustVector<T>& user, int N,
                                 std::vector<double> similarities) {
    static_assert(std::is_same<T, double>::value, "lshkm_compat::get_top_N_recom matches CustVector<double> only");
    const size_t n = neighbors.size(), d = user.getDimensions()->size();
    const std::vector<int> unk = user.getUnknownIndexes();
    std::vector<int> out(N > 0 ? N : 0, 0);
    if (N <= 0) return out;
    if (similarities.size() < n) throw std::invalid_argument("lshkm_compat: fewer similarities than neighbours");
    const size_t rows = n > 0 ? n : 1;
    std::vector<double> X(rows * d, 0.0), xm(rows, 0.0);
    for (size_t i = 0; i < n; i++) {
        const std::vector<T>& x = *neighbors[i]->getDimensions();
        for (size_t j = 0; j < d && j < x.size(); j++) X[i * d + j] = x[j];
        xm[i] = neighbors[i]->getKnownMean();
    }
    const int P = n > 0 ? (int)n : 1;
    std::vector<int32_t> nb(P, 0), cnt = {(int32_t)n};
    std::vector<double> sm(P, 0.0);
    for (size_t i = 0; i < n; i++) { nb[i] = (int32_t)i; sm[i] = similarities[i]; }
    std::vector<int64_t> up = {0, (int64_t)unk.size()};
    std::vector<int32_t> ui(unk.begin(), unk.end());
    if (ui.empty()) ui.push_back(0);
    const double um = user.getKnownMean();
    DevMem Xd = upload(X.data(), X.size()), xmd = upload(xm.data(), rows), umd = upload(&um, 1);
    DevMem upd = upload(up.data(), 2), uid = upload(ui.data(), ui.size());
    DevMem nbd = upload(nb.data(), nb.size()), smd = upload(sm.data(), sm.size()), cnd = upload(cnt.data(), 1);
    DevMem od(sizeof(int32_t) * N);
    check(lshkm_top_n_recom(context(), Xd.as<double>(), xmd.as<double>(), (int64_t)rows, (int)d, umd.as<double>(), 1,
                            upd.as<int64_t>(), uid.as<int32_t>(), nbd.as<int32_t>(), smd.as<double>(),
                            cnd.as<int32_t>(), P, N, od.as<int32_t>()));
    std::vector<int32_t> o(N);
    download(o.data(), od, N);
    for (int i = 0; i < N; i++) out[i] = o[i];
    return out;
}

// The 3-argument overload's clusters, kept on the device per thread. main.cpp
// calls it once per user with a copy of that user's whole cluster
// (main.cpp:260-269, :353-373): each cluster is marshalled and uploaded once,
// and a later call with the same neighbour list only compares it with the
// cached copy (pointers, known means and every value, memcmp -- O(cluster)
// reads and no upload); any difference re-marshals it, so results never come
// from stale data. Entries past LSHKM_COMPAT_CLUSTER_CACHE bytes of host copies
// are dropped (the whole cache is cleared).
#ifndef LSHKM_COMPAT_CLUSTER_CACHE
#define LSHKM_COMPAT_CLUSTER_CACHE (size_t(2) << 30)
#endif
struct ClusterEntry {
    std::vector<const void*> ptrs;
    std::vector<double> X, xm;
    DevMem Xd, xmd, crd, crsd;
};
struct ClusterCache {
    std::unordered_map<uint64_t, ClusterEntry> map;
    size_t bytes = 0;
    uint64_t hits = 0, misses = 0;
};
inline ClusterCache& cluster_cache() {
    (void)context();                 // constructed first, so destroyed after the cache's device buffers
    static thread_local ClusterCache c;
    return c;
}

template <typename T>
const ClusterEntry& cluster_entry(const std::vector<CustVector<T>*>& neighbors, size_t d) {
    const size_t n = neighbors.size();
    uint64_t key = 1469598103934665603ull ^ (uint64_t)d;
    for (auto p : neighbors) key = (key ^ (uint64_t)(uintptr_t)p) * 1099511628211ull;
    ClusterCache& cc = cluster_cache();
    auto it = cc.map.find(key);
    if (it != cc.map.end()) {
        const ClusterEntry& e = it->second;
        bool same = e.ptrs.size() == n && e.X.size() == n * d;
        for (size_t i = 0; same && i < n; i++) {
            const std::vector<T>& x = *neighbors[i]->getDimensions();
            const double m = neighbors[i]->getKnownMean();
            same = e.ptrs[i] == (const void*)neighbors[i] && x.size() == d &&
                   std::memcmp(x.data(), &e.X[i * d], d * sizeof(double)) == 0 &&
                   std::memcmp(&m, &e.xm[i], sizeof(double)) == 0;
        }
        if (same) {
            cc.hits++;
            return e;
        }
        cc.bytes -= e.X.size() * sizeof(double);
        cc.map.erase(it);
    }
    cc.misses++;
    ClusterEntry e;
    e.ptrs.resize(n);
    e.X.resize(n * d);
    e.xm.resize(n);
    for (size_t i = 0; i < n; i++) {
        const std::vector<T>& x = *neighbors[i]->getDimensions();
        if (x.size() != d) throw std::invalid_argument("lshkm_compat: neighbour dimension mismatch");
        for (size_t j = 0; j < d; j++) e.X[i * d + j] = x[j];
        e.xm[i] = neighbors[i]->getKnownMean();
        e.ptrs[i] = neighbors[i];
    }
    // the neighbours as one cluster of an n-row pool, in their order
    std::vector<int64_t> crow = {0, (int64_t)n};
    std::vector<int32_t> crows(n);
    for (size_t i = 0; i < n; i++) crows[i] = (int32_t)i;
    e.Xd = upload(e.X.data(), e.X.size());
    e.xmd = upload(e.xm.data(), n);
    e.crd = upload(crow.data(), 2);
    e.crsd = upload(crows.data(), n);
    if (cc.bytes + e.X.size() * sizeof(double) > LSHKM_COMPAT_CLUSTER_CACHE) {
        cc.map.clear();
        cc.bytes = 0;
    }
    cc.bytes += e.X.size() * sizeof(double);
    return cc.map.emplace(key, std::move(e)).first->second;
}

// get_top_N_recom(neighbors, user, N) -- the 3-argument overload
// (crypto_rec.hpp:327-345) the clustering recommenders call with a whole
// cluster (main.cpp:266, :370): similarities to every neighbour in order,
// predictions over all of them, the quicksort, first N (0-padded).
template <typename T>
std::vector<int> get_top_N_recom(std::vector<CustVector<T>*>& neighbors, CustVector<T>& user, int N) {
    static_assert(std::is_same<T, double>::value, "lshkm_compat::get_top_N_recom matches CustVector<double> only");
    const size_t n = neighbors.size(), d = user.getDimensions()->size();
    if (N <= 0) return std::vector<int>();
    // no neighbours: every prediction is 0/0 (the 4-argument path computes the
    // same sums over an empty list)
    if (n == 0) return lshkm_compat::get_top_N_recom<T>(neighbors, user, N, std::vector<double>());
    const ClusterEntry& ce = cluster_entry(neighbors, d);
    std::vector<int32_t> ucl = {0};
    const std::vector<int> unk = user.getUnknownIndexes();
    for (int e : unk)
        if (e < 0 || (size_t)e >= d) throw std::out_of_range("lshkm_compat: unknown index outside the vector");
    std::vector<int64_t> up = {0, (int64_t)unk.size()};
    std::vector<int32_t> ui(unk.begin(), unk.end());
    if (ui.empty()) ui.push_back(0);
    const double um = user.getKnownMean();
    DevMem Ud = upload(user.getDimensions()->data(), d);
    DevMem umd = upload(&um, 1), ucd = upload(ucl.data(), 1);
    DevMem upd = upload(up.data(), 2), uid = upload(ui.data(), ui.size());
    DevMem od(sizeof(int32_t) * N);
    check(lshkm_cluster_top_n_f64(context(), ce.Xd.as<double>(), ce.xmd.as<double>(), (int64_t)n, (int)d,
                                  ce.crd.as<int64_t>(), ce.crsd.as<int32_t>(), 1, Ud.as<double>(), umd.as<double>(), 1,
                                  ucd.as<int32_t>(), upd.as<int64_t>(), uid.as<int32_t>(), N, od.as<int32_t>()));
    std::vector<int32_t> o(N);
    download(o.data(), od, N);
    return std::vector<int>(o.begin(), o.end());
}

}  // namespace lshkm_compat

#endif  // LSHKM_COMPAT_HPP
