// ref_harness.cpp — runs the REFERENCE's own hot-path code to produce golden
// fixtures and the CPU baseline. TEST INFRASTRUCTURE ONLY: nothing in the
// product links or calls this.
//
// Built by oracle/Makefile from this file plus the reference's sources where
// they lie (/root/reference/lib/*.hpp by include path, utils.cpp, tweet.cpp),
// with g++ -O0 as the reference ships (-O1/-O2 crash on the UB at
// cust_hashtable.hpp:65-70; clang changes M at euclidean_phi_gen.hpp:70).
// The binary goes to oracle/_ref/ only (git-ignored).
//
// Determinism: the reference seeds every RNG from system_clock::now()
// (lsh_cube.hpp:49-51,112-114; initialization.hpp:42-44,75-77). We interpose
// std::chrono::_V2::system_clock::now() at link time and return g_seed ticks.
//
// Output: .npy files (little endian) into an output directory.

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <map>
#include <random>
#include <set>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

static long long g_seed = 12345;

namespace std { namespace chrono { inline namespace _V2 {
system_clock::time_point system_clock::now() noexcept {
    return system_clock::time_point(system_clock::duration(g_seed));
}
}}}

// Read generator internals (params, memo tables). Std headers are already in.
#define private public
#include "utils.hpp"
#include "lsh_cube.hpp"
#include "clustering_phases/assignment.hpp"
#include "clustering_phases/update.hpp"
#include "clustering_phases/initialization.hpp"
#include "crypto_rec.hpp"
#include "clustering_phases/silhouette.hpp"
#include "in_out/vector_reader.hpp"
#include "in_out/arg_parser.h"
#undef private

#include "../include/lshkm_synth.h"

typedef CustVector<double> Vec;

// ---------------------------------------------------------------- npy writer
template <typename T> struct NpyType;
template <> struct NpyType<float>   { static const char* s() { return "<f4"; } };
template <> struct NpyType<double>  { static const char* s() { return "<f8"; } };
template <> struct NpyType<int32_t> { static const char* s() { return "<i4"; } };
template <> struct NpyType<int64_t> { static const char* s() { return "<i8"; } };
template <> struct NpyType<uint32_t>{ static const char* s() { return "<u4"; } };
template <> struct NpyType<uint8_t> { static const char* s() { return "|u1"; } };

template <typename T>
static void write_npy(const std::string& path, const std::vector<T>& data, const std::vector<size_t>& shape) {
    std::string hdr = std::string("{'descr': '") + NpyType<T>::s() + "', 'fortran_order': False, 'shape': (";
    for (size_t i = 0; i < shape.size(); i++) hdr += std::to_string(shape[i]) + (shape.size() == 1 ? ",)" : (i + 1 < shape.size() ? ", " : ")"));
    if (shape.empty()) hdr += ")";
    hdr += ", }";
    size_t total = 10 + hdr.size() + 1;
    size_t pad = (64 - total % 64) % 64;
    hdr += std::string(pad, ' ') + "\n";
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) { fprintf(stderr, "cannot write %s\n", path.c_str()); exit(2); }
    unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
    fwrite(magic, 1, 8, f);
    uint16_t hl = (uint16_t)hdr.size();
    fwrite(&hl, 2, 1, f);
    fwrite(hdr.data(), 1, hdr.size(), f);
    if (!data.empty()) fwrite(data.data(), sizeof(T), data.size(), f);
    fclose(f);
}

static std::vector<float> read_f32(const std::string& path, size_t count) {
    std::vector<float> v(count);
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) { fprintf(stderr, "cannot read %s\n", path.c_str()); exit(2); }
    if (fread(v.data(), sizeof(float), count, f) != count) { fprintf(stderr, "short read %s\n", path.c_str()); exit(2); }
    fclose(f);
    return v;
}

static std::vector<double> read_f64(const std::string& path, size_t count) {
    std::vector<double> v(count);
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) { fprintf(stderr, "cannot read %s\n", path.c_str()); exit(2); }
    if (fread(v.data(), sizeof(double), count, f) != count) { fprintf(stderr, "short read %s\n", path.c_str()); exit(2); }
    fclose(f);
    return v;
}

template <typename T>
static std::vector<T> read_raw(const std::string& path, size_t count) {
    std::vector<T> v(count);
    if (count == 0) return v;
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) { fprintf(stderr, "cannot read %s\n", path.c_str()); exit(2); }
    if (fread(v.data(), sizeof(T), count, f) != count) { fprintf(stderr, "short read %s\n", path.c_str()); exit(2); }
    fclose(f);
    return v;
}

// Input rows: a ".f64" file holds doubles (general values, the `_f64` paths),
// anything else fp32 values, widened exactly into the reference's doubles.
static std::vector<double> read_rows(const std::string& path, size_t count) {
    if (path.size() > 4 && path.compare(path.size() - 4, 4, ".f64") == 0) return read_f64(path, count);
    std::vector<float> x = read_f32(path, count);
    return std::vector<double>(x.begin(), x.end());
}

template <typename T>
static std::vector<Vec> make_vectors(const std::vector<T>& x, int N, int d, const std::string& prefix) {
    std::vector<Vec> vecs;
    vecs.reserve(N);
    for (int i = 0; i < N; i++) {
        std::vector<double> dims(d);
        for (int j = 0; j < d; j++) dims[j] = (double)x[(size_t)i * d + j];
        vecs.emplace_back(prefix + std::to_string(i), dims);
    }
    return vecs;
}

static std::vector<int> split_ints(const std::string& s) {
    std::vector<int> out;
    std::stringstream ss(s);
    std::string tok;
    while (std::getline(ss, tok, ',')) if (!tok.empty()) out.push_back(std::stoi(tok));
    return out;
}

static void csr_write(const std::string& dir, const std::string& name,
                      const std::vector<std::vector<int32_t>>& lists) {
    std::vector<int64_t> ptr(1, 0);
    std::vector<int32_t> idx;
    for (auto& l : lists) { idx.insert(idx.end(), l.begin(), l.end()); ptr.push_back((int64_t)idx.size()); }
    write_npy(dir + "/" + name + "_ptr.npy", ptr, {ptr.size()});
    write_npy(dir + "/" + name + "_idx.npy", idx, {idx.size()});
}

static std::vector<int32_t> to_indices(const std::vector<Vec*>& ptrs, Vec* base) {
    std::vector<int32_t> out;
    out.reserve(ptrs.size());
    for (auto p : ptrs) out.push_back((int32_t)(p - base));
    return out;
}

// ------------------------------------------------------------------ LSH mode
// lsh IN N d metric k L div w seed OUT [QIN Q NQROWS]
static int mode_lsh(int argc, char** argv) {
    if (argc < 11) { fprintf(stderr, "usage: lsh IN N d metric k L div w seed OUT [QIN Q NQROWS]\n"); return 2; }
    std::string in = argv[1]; int N = atoi(argv[2]); int d = atoi(argv[3]);
    std::string metric = argv[4]; int k = atoi(argv[5]); int L = atoi(argv[6]);
    int div = atoi(argv[7]); double w = atof(argv[8]); g_seed = atoll(argv[9]);
    std::string out = argv[10];
    std::vector<double> x = read_rows(in, (size_t)N * d);
    std::vector<Vec> vecs = make_vectors(x, N, d, "");

    std::vector<CustHashtable<double>*> tables = create_LSH_hashtables<double>(vecs, metric, k, L, div, w);
    int nb = (metric == "euclidean") ? N / div : (int)pow(2, k);

    std::vector<int32_t> tuples, phi((size_t)N * L), bucket((size_t)N * L);
    std::vector<float> V, T, W; std::vector<int32_t> R; std::vector<double> RC;
    for (int l = 0; l < L; l++) {
        HashGenerator<double>* g = tables[l]->hashGenerator;
        if (metric == "euclidean") {
            auto* pg = dynamic_cast<EuclideanPhiGen<double>*>(g);
            for (int i = 0; i < k; i++) {
                auto* h = pg->hFunctions[i];
                for (int j = 0; j < d; j++) V.push_back((*h->v->getDimensions())[j]);
                T.push_back(h->t); W.push_back(h->w); R.push_back(pg->rs[i]);
            }
        } else {
            auto* cg = dynamic_cast<CosineGGen<double>*>(g);
            for (int i = 0; i < k; i++)
                for (int j = 0; j < d; j++) RC.push_back((*cg->hFunctions[i]->r->getDimensions())[j]);
        }
    }
    if (metric == "euclidean") {
        tuples.resize((size_t)N * L * k);
        for (int n = 0; n < N; n++)
            for (int l = 0; l < L; l++) {
                auto* pg = dynamic_cast<EuclideanPhiGen<double>*>(tables[l]->hashGenerator);
                std::vector<int>& t = pg->id_to_det_hashes[vecs[n].getId()];
                for (int i = 0; i < k; i++) tuples[((size_t)n * L + l) * k + i] = t[i];
            }
    }
    for (int n = 0; n < N; n++)
        for (int l = 0; l < L; l++) {
            phi[(size_t)n * L + l] = tables[l]->hashGenerator->generate(&vecs[n]);
            bucket[(size_t)n * L + l] = tables[l]->getHash(&vecs[n]);
        }
    std::vector<std::vector<int32_t>> members;
    for (int l = 0; l < L; l++)
        for (int b = 0; b < nb; b++) members.push_back(to_indices(tables[l]->getBucketFromIndex(b), vecs.data()));

    if (metric == "euclidean") {
        write_npy(out + "/V.npy", V, {(size_t)L, (size_t)k, (size_t)d});
        write_npy(out + "/t.npy", T, {(size_t)L, (size_t)k});
        write_npy(out + "/w.npy", W, {(size_t)L, (size_t)k});
        write_npy(out + "/r.npy", R, {(size_t)L, (size_t)k});
        write_npy(out + "/tuples.npy", tuples, {(size_t)N, (size_t)L, (size_t)k});
    } else {
        write_npy(out + "/R.npy", RC, {(size_t)L, (size_t)k, (size_t)d});
    }
    write_npy(out + "/phi.npy", phi, {(size_t)N, (size_t)L});
    write_npy(out + "/bucket.npy", bucket, {(size_t)N, (size_t)L});
    csr_write(out, "members", members);

    // Queries: NQROWS dataset rows (in row order), then Q external vectors.
    if (argc >= 14) {
        std::string qin = argv[11]; int Q = atoi(argv[12]); int nqrows = atoi(argv[13]);
        std::vector<double> qx = read_rows(qin, (size_t)Q * d);
        std::vector<Vec> qvecs = make_vectors(qx, Q, d, "q");
        std::vector<std::vector<int32_t>> filt, unf;
        for (int r = 0; r < nqrows + Q; r++) {
            Vec* q = r < nqrows ? &vecs[r] : &qvecs[r - nqrows];
            filt.push_back(to_indices(get_LSH_filtered_combined_buckets(tables, q), vecs.data()));
            unf.push_back(to_indices(get_LSH_combined_buckets(tables, q), vecs.data()));
        }
        csr_write(out, "qfilt", filt);
        csr_write(out, "qunf", unf);
    }
    for (auto t : tables) delete t;
    return 0;
}

// ----------------------------------------------------------------- cube mode
// cube IN N d metric k w seed PROBES_CSV OUT [QIN Q NQROWS]
static int mode_cube(int argc, char** argv) {
    if (argc < 9) { fprintf(stderr, "usage: cube IN N d metric k w seed PROBES OUT [QIN Q NQROWS]\n"); return 2; }
    std::string in = argv[1]; int N = atoi(argv[2]); int d = atoi(argv[3]);
    std::string metric = argv[4]; int k = atoi(argv[5]); double w = atof(argv[6]);
    g_seed = atoll(argv[7]); std::vector<int> probes = split_ints(argv[8]);
    std::string out = argv[9];
    std::vector<double> x = read_rows(in, (size_t)N * d);
    std::vector<Vec> vecs = make_vectors(x, N, d, "");

    CustHashtable<double>* cube = create_hypercube<double>(vecs, metric, k, w);
    auto* hg = dynamic_cast<HypercubeGen<double>*>(cube->hashGenerator);
    int nb = 1 << k;

    std::vector<float> V, T, W; std::vector<double> RC;
    std::vector<int32_t> memo_f, memo_h, memo_bit;
    for (int i = 0; i < k; i++) {
        if (metric == "euclidean") {
            auto* fg = dynamic_cast<EuclideanFGen<double>*>(hg->fFunctions[i]);
            for (int j = 0; j < d; j++) V.push_back((*fg->hGenerator->v->getDimensions())[j]);
            T.push_back(fg->hGenerator->t); W.push_back(fg->hGenerator->w);
            std::map<int, int> sorted(fg->num_to_bin_hashes.begin(), fg->num_to_bin_hashes.end());
            for (auto& kv : sorted) { memo_f.push_back(i); memo_h.push_back(kv.first); memo_bit.push_back(kv.second); }
        } else {
            auto* ch = dynamic_cast<CosineHGen<double>*>(hg->fFunctions[i]);
            for (int j = 0; j < d; j++) RC.push_back((*ch->r->getDimensions())[j]);
        }
    }
    std::vector<int32_t> vertex(N), hvals;
    for (int n = 0; n < N; n++) vertex[n] = cube->getHash(&vecs[n]);   // all h already seen: no draws
    if (metric == "euclidean") {
        for (int n = 0; n < N; n++)
            for (int i = 0; i < k; i++)
                hvals.push_back(dynamic_cast<EuclideanFGen<double>*>(hg->fFunctions[i])->hGenerator->generate(&vecs[n]));
    }
    std::vector<std::vector<int32_t>> members;
    for (int b = 0; b < nb; b++) members.push_back(to_indices(cube->getBucketFromIndex(b), vecs.data()));

    if (metric == "euclidean") {
        write_npy(out + "/V.npy", V, {(size_t)k, (size_t)d});
        write_npy(out + "/t.npy", T, {(size_t)k});
        write_npy(out + "/w.npy", W, {(size_t)k});
        write_npy(out + "/memo_f.npy", memo_f, {memo_f.size()});
        write_npy(out + "/memo_h.npy", memo_h, {memo_h.size()});
        write_npy(out + "/memo_bit.npy", memo_bit, {memo_bit.size()});
        write_npy(out + "/h.npy", hvals, {(size_t)N, (size_t)k});
    } else {
        write_npy(out + "/R.npy", RC, {(size_t)k, (size_t)d});
    }
    write_npy(out + "/vertex.npy", vertex, {(size_t)N});
    csr_write(out, "members", members);
    write_npy(out + "/probes.npy", std::vector<int32_t>(probes.begin(), probes.end()), {probes.size()});

    // Queries. The F-coin engine is a local of create_hypercube (lsh_cube.hpp:113)
    // held by pointer in every EuclideanFGen (euclidean_f_gen.hpp:58): a query
    // whose h was never seen draws from a dead stack frame (UB). Such queries are
    // skipped here and marked in qmask; only fully-seen queries are pinned.
    if (argc >= 13) {
        std::string qin = argv[10]; int Q = atoi(argv[11]); int nqrows = atoi(argv[12]);
        std::vector<double> qx = read_rows(qin, (size_t)Q * d);
        std::vector<Vec> qvecs = make_vectors(qx, Q, d, "q");
        std::vector<uint8_t> qmask;
        std::vector<Vec*> qs;
        for (int r = 0; r < nqrows + Q; r++) {
            Vec* q = r < nqrows ? &vecs[r] : &qvecs[r - nqrows];
            bool seen = true;
            if (metric == "euclidean")
                for (int i = 0; i < k; i++) {
                    auto* fg = dynamic_cast<EuclideanFGen<double>*>(hg->fFunctions[i]);
                    if (fg->num_to_bin_hashes.count(fg->hGenerator->generate(q)) == 0) seen = false;
                }
            qmask.push_back(seen ? 1 : 0);
            if (seen) qs.push_back(q);
        }
        write_npy(out + "/qmask.npy", qmask, {qmask.size()});
        for (int p : probes) {
            std::vector<std::vector<int32_t>> res;
            for (Vec* q : qs) res.push_back(to_indices(get_hypercube_combined_buckets(*cube, q, p, k), vecs.data()));
            csr_write(out, "q_probes" + std::to_string(p), res);
        }
    }
    delete cube;
    return 0;
}

// ---------------------------------------------------------------- lloyd mode
// lloyd IN N d K metric iters min_dist OUT [CENTERS_F64 | -]  [rows_csv]
// Initial centroids: dataset rows i*(N/K) (or rows_csv), or an fp64 file of
// K*d external centers (ids "c<i>", not dataset rows).
static int mode_lloyd(int argc, char** argv) {
    if (argc < 9) { fprintf(stderr, "usage: lloyd IN N d K metric iters min_dist OUT [CENTERS|-] [rows]\n"); return 2; }
    std::string in = argv[1]; int N = atoi(argv[2]); int d = atoi(argv[3]); int K = atoi(argv[4]);
    std::string metric = argv[5]; int iters = atoi(argv[6]); double min_dist = atof(argv[7]);
    std::string out = argv[8];
    std::vector<double> x = read_rows(in, (size_t)N * d);
    std::vector<Vec> vecs = make_vectors(x, N, d, "");
    std::vector<Vec*> centroids(K);
    std::vector<Vec> ext;
    std::vector<int32_t> src_rows(K, -1);
    if (argc >= 10 && std::string(argv[9]) != "-") {
        std::vector<double> c = read_f64(argv[9], (size_t)K * d);
        ext.reserve(K);
        for (int i = 0; i < K; i++) ext.emplace_back("c" + std::to_string(i), std::vector<double>(c.begin() + (size_t)i * d, c.begin() + (size_t)(i + 1) * d));
        for (int i = 0; i < K; i++) centroids[i] = &ext[i];
    } else {
        std::vector<int> rows;
        if (argc >= 11) rows = split_ints(argv[10]);
        for (int i = 0; i < K; i++) {
            int r = rows.empty() ? i * (N / K) : rows[i];
            centroids[i] = &vecs[r]; src_rows[i] = r;
        }
    }
    write_npy(out + "/src_rows.npy", src_rows, {(size_t)K});
    std::vector<double> c0;
    for (int c = 0; c < K; c++) for (int j = 0; j < d; j++) c0.push_back((*centroids[c]->getDimensions())[j]);
    write_npy(out + "/centers0.npy", c0, {(size_t)K, (size_t)d});

    bool cont = true; int it = 0;
    std::vector<int32_t> flags;
    while (cont && it < iters) {
        lloyds_assignment(vecs, centroids, metric);
        std::vector<int32_t> assign(N); std::vector<double> dist(N);
        for (int n = 0; n < N; n++) { assign[n] = vecs[n].getCluster(); dist[n] = vecs[n].getDistFromCentroid(); }
        write_npy(out + "/assign" + std::to_string(it) + ".npy", assign, {(size_t)N});
        write_npy(out + "/dist" + std::to_string(it) + ".npy", dist, {(size_t)N});
        // silhouette_cluster (silhouette.hpp:31-80) of this assignment
        std::vector<double> sil = silhouette_cluster(separate_clusters_from_input(vecs, K), centroids, metric);
        write_npy(out + "/sil" + std::to_string(it) + ".npy", sil, {sil.size()});
        cont = k_means(vecs, centroids, metric, min_dist);
        flags.push_back(cont ? 1 : 0);
        std::vector<double> cs;
        for (int c = 0; c < K; c++) for (int j = 0; j < d; j++) cs.push_back((*centroids[c]->getDimensions())[j]);
        write_npy(out + "/centers" + std::to_string(it + 1) + ".npy", cs, {(size_t)K, (size_t)d});
        it++;
    }
    write_npy(out + "/cont.npy", flags, {flags.size()});
    for (auto c : centroids) if (c->getId() == "k_means_center") delete c;
    return 0;
}

// ------------------------------------------------------------ kmeanspp mode
// kmeanspp IN N d K metric seed OUT  — k-means++ seeding (initialization.hpp:71-156)
static int mode_kmeanspp(int argc, char** argv) {
    if (argc < 8) { fprintf(stderr, "usage: kmeanspp IN N d K metric seed OUT\n"); return 2; }
    std::string in = argv[1]; int N = atoi(argv[2]); int d = atoi(argv[3]); int K = atoi(argv[4]);
    std::string metric = argv[5]; g_seed = atoll(argv[6]); std::string out = argv[7];
    std::vector<double> x = read_rows(in, (size_t)N * d);
    std::vector<Vec> vecs = make_vectors(x, N, d, "");
    std::vector<Vec*> c = k_means_pp(vecs, K, metric);
    std::vector<Vec*> r = rand_selection(vecs, K);
    std::vector<int32_t> rows, rrows;
    for (auto p : c) rows.push_back((int32_t)(p - vecs.data()));
    for (auto p : r) rrows.push_back((int32_t)(p - vecs.data()));
    write_npy(out + "/kpp_rows.npy", rows, {rows.size()});
    write_npy(out + "/rand_rows.npy", rrows, {rrows.size()});
    return 0;
}

// ------------------------------------------------------------ recom mode
// recom DIR N d Q P NTOP — the recommend step (crypto_rec.hpp:213-345) as main.cpp
// uses it (:160-168): per user, get_P_closest over its candidate neighbours, then
// get_top_N_recom with those similarities. DIR holds x.f64 [N][d], xmean.f64
// [N], u.f64 [Q][d], umean.f64 [Q], unk_ptr.i64 / unk_idx.i32 (each user's
// unknown indexes), cand_ptr.i64 / cand_idx.i32 (neighbour rows, in order).
// Outputs into DIR: pc_idx [Q][P] (-1 pad), pc_sim [Q][P] (0 pad), pc_cnt [Q],
// top [Q][NTOP] (-1 for users without neighbours, which main.cpp skips).
static int mode_recom(int argc, char** argv) {
    if (argc < 7) { fprintf(stderr, "usage: recom DIR N d Q P NTOP\n"); return 2; }
    std::string dir = argv[1];
    int N = atoi(argv[2]), d = atoi(argv[3]), Q = atoi(argv[4]), P = atoi(argv[5]), NT = atoi(argv[6]);
    std::vector<double> x = read_raw<double>(dir + "/x.f64", (size_t)N * d);
    std::vector<double> xm = read_raw<double>(dir + "/xmean.f64", N);
    std::vector<double> u = read_raw<double>(dir + "/u.f64", (size_t)Q * d);
    std::vector<double> um = read_raw<double>(dir + "/umean.f64", Q);
    std::vector<int64_t> up = read_raw<int64_t>(dir + "/unk_ptr.i64", Q + 1);
    std::vector<int32_t> ui = read_raw<int32_t>(dir + "/unk_idx.i32", (size_t)up[Q]);
    std::vector<int64_t> cp = read_raw<int64_t>(dir + "/cand_ptr.i64", Q + 1);
    std::vector<int32_t> ci = read_raw<int32_t>(dir + "/cand_idx.i32", (size_t)cp[Q]);
    std::vector<Vec> pool;
    pool.reserve(N);
    for (int i = 0; i < N; i++)
        pool.emplace_back("p" + std::to_string(i), std::vector<double>(x.begin() + (size_t)i * d, x.begin() + (size_t)(i + 1) * d),
                          std::set<int>(), xm[i]);
    std::vector<int32_t> pc_idx((size_t)Q * P, -1), pc_cnt(Q, 0), top((size_t)Q * NT, -1);
    std::vector<double> pc_sim((size_t)Q * P, 0.0);
    for (int q = 0; q < Q; q++) {
        std::set<int> unk(ui.begin() + up[q], ui.begin() + up[q + 1]);
        Vec user("u" + std::to_string(q), std::vector<double>(u.begin() + (size_t)q * d, u.begin() + (size_t)(q + 1) * d),
                 unk, um[q]);
        std::vector<Vec*> nb;
        for (int64_t e = cp[q]; e < cp[q + 1]; e++) nb.push_back(&pool[ci[e]]);
        if (nb.empty()) continue;
        std::vector<double> sims = get_P_closest(nb, user, P);
        for (size_t i = 0; i < nb.size(); i++) {
            pc_idx[(size_t)q * P + i] = (int32_t)(nb[i] - pool.data());
            pc_sim[(size_t)q * P + i] = sims[i];
        }
        pc_cnt[q] = (int32_t)nb.size();
        std::vector<int> t = get_top_N_recom(nb, user, NT, sims);
        for (int i = 0; i < NT; i++) top[(size_t)q * NT + i] = t[i];
    }
    write_npy(dir + "/pc_idx.npy", pc_idx, {(size_t)Q, (size_t)P});
    write_npy(dir + "/pc_sim.npy", pc_sim, {(size_t)Q, (size_t)P});
    write_npy(dir + "/pc_cnt.npy", pc_cnt, {(size_t)Q});
    write_npy(dir + "/top.npy", top, {(size_t)Q, (size_t)NT});
    return 0;
}

// --------------------------------------------------------------- bench mode
// bench NH NA K seed — the reference's own CPU path on synthetic data, one
// thread, as shipped (-O0). Prints one JSON line.
static int mode_bench(int argc, char** argv) {
    if (argc < 5) { fprintf(stderr, "usage: bench NH NA K seed\n"); return 2; }
    int NH = atoi(argv[1]); int NA = atoi(argv[2]); int K = atoi(argv[3]); uint64_t seed = strtoull(argv[4], 0, 10);
    const int d = 128;
    int NX = NH > NA ? NH : NA;
    std::vector<float> x((size_t)NX * d);
    for (size_t i = 0; i < (size_t)NX; i++)
        for (int j = 0; j < d; j++) x[i * d + j] = lshkm_synth_value(seed, i, d, j);
    std::vector<Vec> vh = make_vectors(std::vector<float>(x.begin(), x.begin() + (size_t)NH * d), NH, d, "");
    std::vector<Vec> va = make_vectors(std::vector<float>(x.begin(), x.begin() + (size_t)NA * d), NA, d, "");
    g_seed = 12345;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<CustHashtable<double>*> tables = create_LSH_hashtables<double>(vh, "euclidean", 4, 5, 100, 0.4);
    auto t1 = std::chrono::steady_clock::now();
    std::vector<Vec*> cents(K);
    for (int i = 0; i < K; i++) cents[i] = &va[i * (NA / K)];
    auto t2 = std::chrono::steady_clock::now();
    lloyds_assignment(va, cents, std::string("euclidean"));
    auto t3 = std::chrono::steady_clock::now();
    double th = std::chrono::duration<double>(t1 - t0).count();
    double ta = std::chrono::duration<double>(t3 - t2).count();
    printf("{\"hash_pts\": %d, \"hash_s\": %.6f, \"assign_pts\": %d, \"assign_s\": %.6f, \"K\": %d}\n", NH, th, NA, ta, K);
    for (auto t : tables) delete t;
    return 0;
}

// ------------------------------------------------------------- range mode
// range IN N d K metric family k L div w probes iters min_dist seed OUT
// lsh_range_assignment / cube_range_assignment (assignment.hpp:108-145) with
// centroids = rows i*(N/K), then k_means (update.hpp:37-86), `iters` times.
// Per iteration: the combined buckets of each centroid (comb<it>_ptr/idx,
// lsh_cube.hpp:77-90 / :139-177, computed before the call as the call does),
// assign<it>/dist<it>, centers<it> (the centroids used). The cube family is
// only pinned at iteration 0 (later centers may hash to unseen h, whose coins
// come from a dead engine, lsh_cube.hpp:113).
static int mode_range(int argc, char** argv) {
    if (argc < 16) { fprintf(stderr, "usage: range IN N d K metric family k L div w probes iters min_dist seed OUT\n"); return 2; }
    std::string in = argv[1]; int N = atoi(argv[2]); int d = atoi(argv[3]); int K = atoi(argv[4]);
    std::string metric = argv[5], family = argv[6];
    int k = atoi(argv[7]), L = atoi(argv[8]), div = atoi(argv[9]); double w = atof(argv[10]);
    int probes = atoi(argv[11]), iters = atoi(argv[12]); double min_dist = atof(argv[13]);
    g_seed = atoll(argv[14]); std::string out = argv[15];
    std::vector<double> x = read_rows(in, (size_t)N * d);
    std::vector<Vec> vecs = make_vectors(x, N, d, "");
    std::vector<CustHashtable<double>*> tables;
    CustHashtable<double>* cube = nullptr;
    if (family == "lsh") tables = create_LSH_hashtables<double>(vecs, metric, k, L, div, w);
    else cube = create_hypercube<double>(vecs, metric, k, w);
    std::vector<Vec*> centroids(K);
    std::vector<int32_t> src_rows(K);
    for (int i = 0; i < K; i++) { centroids[i] = &vecs[i * (N / K)]; src_rows[i] = i * (N / K); }
    write_npy(out + "/src_rows.npy", src_rows, {(size_t)K});
    bool cont = true; int it = 0;
    while (cont && it < iters) {
        std::vector<double> cs;
        for (int c = 0; c < K; c++) for (int j = 0; j < d; j++) cs.push_back((*centroids[c]->getDimensions())[j]);
        write_npy(out + "/centers" + std::to_string(it) + ".npy", cs, {(size_t)K, (size_t)d});
        std::vector<int32_t> key(K);
        for (int c = 0; c < K; c++) {
            key[c] = c;
            for (int c2 = 0; c2 < c; c2++) if (centroids[c2]->getId() == centroids[c]->getId()) { key[c] = key[c2]; break; }
        }
        write_npy(out + "/key" + std::to_string(it) + ".npy", key, {(size_t)K});
        std::vector<std::vector<int32_t>> comb;
        for (int c = 0; c < K; c++)
            comb.push_back(to_indices(family == "lsh" ? get_LSH_combined_buckets<double>(tables, centroids[c])
                                                      : get_hypercube_combined_buckets<double>(*cube, centroids[c], probes, k),
                                      vecs.data()));
        csr_write(out, "comb" + std::to_string(it), comb);
        if (family == "lsh") lsh_range_assignment(vecs, tables, centroids, metric);
        else cube_range_assignment(vecs, *cube, centroids, metric, probes, k);
        std::vector<int32_t> assign(N); std::vector<double> dist(N);
        for (int n = 0; n < N; n++) { assign[n] = vecs[n].getCluster(); dist[n] = vecs[n].getDistFromCentroid(); }
        write_npy(out + "/assign" + std::to_string(it) + ".npy", assign, {(size_t)N});
        write_npy(out + "/dist" + std::to_string(it) + ".npy", dist, {(size_t)N});
        // silhouette_cluster (silhouette.hpp:31-80) of this assignment
        std::vector<double> sil = silhouette_cluster(separate_clusters_from_input(vecs, K), centroids, metric);
        write_npy(out + "/sil" + std::to_string(it) + ".npy", sil, {sil.size()});
        cont = k_means(vecs, centroids, metric, min_dist);
        it++;
        if (family != "lsh") break;
    }
    std::vector<int32_t> nit(1, it);
    write_npy(out + "/iters.npy", nit, {1});
    for (auto c : centroids) if (c->getId() == "k_means_center") delete c;
    for (auto t : tables) delete t;
    delete cube;
    return 0;
}

// --------------------------------------------------------------- csv mode
// csv PATH DELIM_ASCII STRT_LINE OUT — VectorReader<double>::read
// (vector_reader.hpp:54-85) with main.cpp:82's stod: ids (bytes + offsets),
// values (the rows must be of equal length here), metadata lines.
static int mode_csv(int argc, char** argv) {
    if (argc < 5) { fprintf(stderr, "usage: csv PATH DELIM_ASCII STRT_LINE OUT\n"); return 2; }
    VectorReader<double> rd(argv[1]);
    const char delim = (char)atoi(argv[2]);
    rd.read(delim, atoi(argv[3]), [](const std::string& x) { return std::stod(x); });
    std::string out = argv[4];
    std::vector<Vec> vs = rd.getReadVectors();
    std::vector<uint8_t> idb; std::vector<int64_t> off(1, 0); std::vector<double> x;
    size_t d = vs.empty() ? 0 : vs[0].getDimensions()->size();
    for (auto& v : vs) {
        std::string id = v.getId();
        idb.insert(idb.end(), id.begin(), id.end());
        off.push_back((int64_t)idb.size());
        if (v.getDimensions()->size() != d) { fprintf(stderr, "ragged\n"); return 3; }
        x.insert(x.end(), v.getDimensions()->begin(), v.getDimensions()->end());
    }
    write_npy(out + "/id_bytes.npy", idb, {idb.size()});
    write_npy(out + "/id_off.npy", off, {off.size()});
    write_npy(out + "/x.npy", x, {vs.size(), d});
    std::vector<uint8_t> mb; std::vector<int64_t> moff(1, 0);
    for (int i = 0; i < atoi(argv[3]) - 1; i++) {
        std::string m = rd.getMetaLine(i);
        mb.insert(mb.end(), m.begin(), m.end());
        moff.push_back((int64_t)mb.size());
    }
    write_npy(out + "/meta_bytes.npy", mb, {mb.size()});
    write_npy(out + "/meta_off.npy", moff, {moff.size()});
    return 0;
}

// -------------------------------------------------------------- conf mode
// conf PATH KEY... — ArgParser(file_to_args(PATH, ' ')) (utils.cpp:53-69,
// arg_parser.cpp:21-33): one line per key, "1 <value>" or "0" when the flag is
// absent or the last token (getFlagValue would build std::string(NULL)).
static int mode_conf(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: conf PATH KEY...\n"); return 2; }
    std::vector<std::string> args = file_to_args(argv[1], ' ');
    ArgParser ap(args);
    for (int i = 2; i < argc; i++) {
        std::string key = argv[i];
        auto it = std::find(args.begin(), args.end(), key);
        if (!ap.flagExists(key) || it + 1 == args.end()) printf("0\n");
        else printf("1 %s\n", ap.getFlagValue(key).c_str());
    }
    return 0;
}

// ---------------------------------------------------------------- c1 mode
// c1 CSV DELIM_ASCII K iters min_dist seed OUT — main.cpp:81-111 (config C1):
// VectorReader<double> + stod, k_means_pp (cosine), then lloyds_assignment +
// k_means until converged or `iters`; writes kpp_rows, assign/centers per
// iteration, iters.
static int mode_c1(int argc, char** argv) {
    if (argc < 8) { fprintf(stderr, "usage: c1 CSV DELIM K iters min_dist seed OUT\n"); return 2; }
    VectorReader<double> rd(argv[1]);
    rd.read((char)atoi(argv[2]), 1, [](const std::string& x) { return std::stod(x); });
    std::vector<Vec> vecs = rd.getReadVectors();
    int K = atoi(argv[3]), iters = atoi(argv[4]); double min_dist = atof(argv[5]);
    g_seed = atoll(argv[6]); std::string out = argv[7];
    const std::string metric = "cosine";
    std::vector<Vec*> centroids = k_means_pp(vecs, K, metric);
    std::vector<int32_t> rows;
    for (auto p : centroids) rows.push_back((int32_t)(p - vecs.data()));
    write_npy(out + "/kpp_rows.npy", rows, {rows.size()});
    int it = 0; bool cont = true;
    while (cont && it < iters) {
        lloyds_assignment(vecs, centroids, metric);
        std::vector<int32_t> assign; std::vector<double> dist;
        for (auto& v : vecs) { assign.push_back(v.getCluster()); dist.push_back(v.getDistFromCentroid()); }
        write_npy(out + "/assign" + std::to_string(it) + ".npy", assign, {assign.size()});
        write_npy(out + "/dist" + std::to_string(it) + ".npy", dist, {dist.size()});
        cont = k_means(vecs, centroids, metric, min_dist);
        std::vector<double> cs;
        for (int c = 0; c < K; c++) for (double x : *centroids[c]->getDimensions()) cs.push_back(x);
        write_npy(out + "/centers" + std::to_string(it + 1) + ".npy", cs, {(size_t)K, cs.size() / K});
        it++;
    }
    std::vector<int32_t> nit(1, it), fl(1, cont ? 1 : 0);
    write_npy(out + "/iters.npy", nit, {1});
    write_npy(out + "/cont.npy", fl, {1});
    for (auto c : centroids) if (c->getId() == "k_means_center") delete c;
    return 0;
}

// ------------------------------------------------------------- chain mode
// chain DIR N Q d k L div w seed P NTOP SELF — the cosine-LSH recommender of
// main.cpp:149-176 (Part A, SELF = 1: the users are the indexed vectors
// themselves) / :186-222 (Part B, SELF = 0: tables over another pool):
// create_LSH_hashtables<double>(pool, "cosine", k, L, div, w), then per user
// get_LSH_filtered_combined_buckets, get_P_closest (P) and get_top_N_recom
// (NTOP), skipping users without neighbours. DIR holds pool.f64 [N][d],
// pmean.f64 [N], punk_ptr.i64 / punk_idx.i32 (the pool's unknown indexes)
// and, for SELF = 0, users.f64 [Q][d], umean.f64, uunk_ptr.i64 / uunk_idx.i32.
// Outputs: R [L][k][d], g [N][L] (bucket of every pool vector), nb_ptr/nb_idx
// (each user's combined bucket, row order), pc_idx/pc_sim [Q][P] (-1 / 0 pad),
// pc_cnt [Q], top [Q][NTOP] (-1 rows for skipped users).
static std::vector<Vec> read_user_vectors(const std::string& dir, const std::string& pre, int N, int d,
                                          const std::string& id) {
    std::vector<double> x = read_raw<double>(dir + "/" + pre + ".f64", (size_t)N * d);
    std::vector<double> m = read_raw<double>(dir + "/" + (pre == "pool" ? std::string("pmean") : std::string("umean")) + ".f64", N);
    const std::string u = pre == "pool" ? "punk" : "uunk";
    std::vector<int64_t> up = read_raw<int64_t>(dir + "/" + u + "_ptr.i64", N + 1);
    std::vector<int32_t> ui = read_raw<int32_t>(dir + "/" + u + "_idx.i32", (size_t)up[N]);
    std::vector<Vec> v;
    v.reserve(N);
    for (int i = 0; i < N; i++)
        v.emplace_back(id + std::to_string(i), std::vector<double>(x.begin() + (size_t)i * d, x.begin() + (size_t)(i + 1) * d),
                       std::set<int>(ui.begin() + up[i], ui.begin() + up[i + 1]), m[i]);
    return v;
}

static int mode_chain(int argc, char** argv) {
    if (argc < 13) { fprintf(stderr, "usage: chain DIR N Q d k L div w seed P NTOP SELF\n"); return 2; }
    std::string dir = argv[1];
    int N = atoi(argv[2]), Q = atoi(argv[3]), d = atoi(argv[4]), k = atoi(argv[5]), L = atoi(argv[6]);
    int div = atoi(argv[7]); double w = atof(argv[8]); g_seed = atoll(argv[9]);
    int P = atoi(argv[10]), NT = atoi(argv[11]); bool self = atoi(argv[12]) != 0;
    std::vector<Vec> pool = read_user_vectors(dir, "pool", N, d, "u");
    std::vector<Vec> others;
    if (!self) others = read_user_vectors(dir, "users", Q, d, "q");
    std::vector<Vec>& users = self ? pool : others;
    if (self) Q = N;
    std::vector<CustHashtable<double>*> tables = create_LSH_hashtables<double>(pool, "cosine", k, L, div, w);
    std::vector<double> RC;
    for (int l = 0; l < L; l++) {
        auto* cg = dynamic_cast<CosineGGen<double>*>(tables[l]->hashGenerator);
        for (int i = 0; i < k; i++)
            for (int j = 0; j < d; j++) RC.push_back((*cg->hFunctions[i]->r->getDimensions())[j]);
    }
    std::vector<int32_t> g((size_t)N * L);
    for (int n = 0; n < N; n++)
        for (int l = 0; l < L; l++) g[(size_t)n * L + l] = tables[l]->getHash(&pool[n]);
    std::vector<std::vector<int32_t>> nbl;
    std::vector<int32_t> pc_idx((size_t)Q * P, -1), pc_cnt(Q, 0), top((size_t)Q * NT, -1);
    std::vector<double> pc_sim((size_t)Q * P, 0.0);
    for (int q = 0; q < Q; q++) {
        Vec& user = users[q];
        std::vector<Vec*> neighbors = get_LSH_filtered_combined_buckets(tables, &user);
        nbl.push_back(to_indices(neighbors, pool.data()));
        if (neighbors.empty()) continue;
        std::vector<double> sims = get_P_closest(neighbors, user, P);
        for (size_t i = 0; i < neighbors.size(); i++) {
            pc_idx[(size_t)q * P + i] = (int32_t)(neighbors[i] - pool.data());
            pc_sim[(size_t)q * P + i] = sims[i];
        }
        pc_cnt[q] = (int32_t)neighbors.size();
        std::vector<int> t = get_top_N_recom(neighbors, user, NT, sims);
        for (int i = 0; i < NT; i++) top[(size_t)q * NT + i] = t[i];
    }
    write_npy(dir + "/R.npy", RC, {(size_t)L, (size_t)k, (size_t)d});
    write_npy(dir + "/g.npy", g, {(size_t)N, (size_t)L});
    csr_write(dir, "nb", nbl);
    write_npy(dir + "/pc_idx.npy", pc_idx, {(size_t)Q, (size_t)P});
    write_npy(dir + "/pc_sim.npy", pc_sim, {(size_t)Q, (size_t)P});
    write_npy(dir + "/pc_cnt.npy", pc_cnt, {(size_t)Q});
    write_npy(dir + "/top.npy", top, {(size_t)Q, (size_t)NT});
    for (auto t : tables) delete t;
    return 0;
}

// -------------------------------------------------------------- crec mode
// crec DIR N F d K iters min_dist seedA seedB NTA NTB — the two clustering
// recommenders of main.cpp, as written:
//   Part A (main.cpp:240-273): rand_selection over the user vectors, Lloyd +
//     k_means (euclidean) until converged or `iters`, separate_clusters_from_input,
//     then per user get_top_N_recom(clusters[user.getCluster()], user, NTA) -- the
//     3-argument overload (crypto_rec.hpp:327-345);
//   Part B (main.cpp:334-381): k_means_pp over the "fake" user vectors, the same
//     loop on them, then per user the nearest centroid by the inline argmin
//     (:356-364) and get_top_N_recom(clusters[argmin], user, NTB), skipping empty
//     clusters.
// DIR holds users.f64 [N][d], umean.f64, uunk_ptr.i64 / uunk_idx.i32 and
// fake.f64 [F][d], fmean.f64, funk_ptr.i64 / funk_idx.i32 (means, unknown sets).
// Outputs: A_rows [K], A_assign [N], A_iters, A_centers [K][d], A_top [N][NTA],
// A_dist [N] (dist_from_centroid after the last Lloyd: fp64 means after the
// first update), A_sim_ptr [N+1] / A_sims (cosineSimilarity(member, user) over
// the user's cluster in member order, as the 3-argument get_top_N_recom forms
// them), A_pred (get_predicted_user_sim at the user's unknown indexes, ascending);
// B_rows [K], B_assign [F], B_iters, B_centers [K][d], B_ucl [N], B_top [N][NTB],
// B_dist [F] (-1 rows for skipped users).
static std::vector<Vec> read_vecs(const std::string& dir, const std::string& pre, int N, int d, const std::string& id) {
    std::vector<double> x = read_raw<double>(dir + "/" + pre + ".f64", (size_t)N * d);
    const std::string a = pre.substr(0, 1);
    std::vector<double> m = read_raw<double>(dir + "/" + a + "mean.f64", N);
    std::vector<int64_t> up = read_raw<int64_t>(dir + "/" + a + "unk_ptr.i64", N + 1);
    std::vector<int32_t> ui = read_raw<int32_t>(dir + "/" + a + "unk_idx.i32", (size_t)up[N]);
    std::vector<Vec> v;
    v.reserve(N);
    for (int i = 0; i < N; i++)
        v.emplace_back(id + std::to_string(i), std::vector<double>(x.begin() + (size_t)i * d, x.begin() + (size_t)(i + 1) * d),
                       std::set<int>(ui.begin() + up[i], ui.begin() + up[i + 1]), m[i]);
    return v;
}

static int mode_crec(int argc, char** argv) {
    if (argc < 12) { fprintf(stderr, "usage: crec DIR N F d K iters min_dist seedA seedB NTA NTB\n"); return 2; }
    std::string dir = argv[1];
    int N = atoi(argv[2]), F = atoi(argv[3]), d = atoi(argv[4]), K = atoi(argv[5]), iters = atoi(argv[6]);
    double min_dist = atof(argv[7]);
    long long seedA = atoll(argv[8]), seedB = atoll(argv[9]);
    int NTA = atoi(argv[10]), NTB = atoi(argv[11]);
    std::vector<Vec> users = read_vecs(dir, "users", N, d, "u");
    std::vector<Vec> fake = read_vecs(dir, "fake", F, d, "f");
    const std::string metric = "euclidean";
    auto centers_of = [&](std::vector<Vec*>& cs) {
        std::vector<double> o;
        for (auto c : cs) o.insert(o.end(), c->getDimensions()->begin(), c->getDimensions()->end());
        return o;
    };
    {   // Part A
        g_seed = seedA;
        std::vector<Vec*> centroids = rand_selection(users, K);
        std::vector<int32_t> rows;
        for (auto p : centroids) rows.push_back((int32_t)(p - users.data()));
        int it = 0;
        bool cont = true;
        while (cont && it < iters) {
            lloyds_assignment(users, centroids, metric);
            cont = k_means(users, centroids, metric, min_dist);
            it++;
        }
        std::vector<std::vector<Vec*>> clusters = separate_clusters_from_input(users, (int)centroids.size());
        std::vector<int32_t> assign(N), top((size_t)N * NTA, -1);
        std::vector<double> dist(N), sims, pred;
        std::vector<int64_t> sim_ptr(1, 0);
        for (int i = 0; i < N; i++) assign[i] = users[i].getCluster();
        for (int i = 0; i < N; i++) dist[i] = users[i].getDistFromCentroid();
        for (int i = 0; i < N; i++) {
            std::vector<Vec*> neighbors = clusters[users[i].getCluster()];
            if (!neighbors.empty()) {
                std::vector<int> t = get_top_N_recom(neighbors, users[i], NTA);
                for (int j = 0; j < NTA; j++) top[(size_t)i * NTA + j] = t[j];
            }
            // the similarities and predictions get_top_N_recom formed (crypto_rec.hpp:327-345)
            std::vector<double> s(neighbors.size());
            for (size_t k = 0; k < neighbors.size(); k++) s[k] = neighbors[k]->cosineSimilarity(&users[i]);
            sims.insert(sims.end(), s.begin(), s.end());
            sim_ptr.push_back((int64_t)sims.size());
            std::vector<double> p = get_predicted_user_sim(neighbors, users[i], s);
            for (int idx : users[i].getUnknownIndexes()) pred.push_back(p[idx]);
        }
        write_npy(dir + "/A_dist.npy", dist, {(size_t)N});
        write_npy(dir + "/A_sim_ptr.npy", sim_ptr, {sim_ptr.size()});
        write_npy(dir + "/A_sims.npy", sims, {sims.size()});
        write_npy(dir + "/A_pred.npy", pred, {pred.size()});
        std::vector<int32_t> nit(1, it);
        write_npy(dir + "/A_rows.npy", rows, {rows.size()});
        write_npy(dir + "/A_assign.npy", assign, {(size_t)N});
        write_npy(dir + "/A_iters.npy", nit, {1});
        write_npy(dir + "/A_centers.npy", centers_of(centroids), {(size_t)K, (size_t)d});
        write_npy(dir + "/A_top.npy", top, {(size_t)N, (size_t)NTA});
        for (auto c : centroids) if (c->getId() == "k_means_center") delete c;
    }
    {   // Part B
        g_seed = seedB;
        std::vector<Vec*> centroids = k_means_pp(fake, K, metric);
        std::vector<int32_t> rows;
        for (auto p : centroids) rows.push_back((int32_t)(p - fake.data()));
        int it = 0;
        bool cont = true;
        while (cont && it < iters) {
            lloyds_assignment(fake, centroids, metric);
            cont = k_means(fake, centroids, metric, min_dist);
            it++;
        }
        std::vector<std::vector<Vec*>> clusters = separate_clusters_from_input(fake, (int)centroids.size());
        std::vector<int32_t> assign(F), ucl(N), top((size_t)N * NTB, -1);
        std::vector<double> fdist(F);
        for (int i = 0; i < F; i++) assign[i] = fake[i].getCluster();
        for (int i = 0; i < F; i++) fdist[i] = fake[i].getDistFromCentroid();
        write_npy(dir + "/B_dist.npy", fdist, {(size_t)F});
        for (int i = 0; i < N; i++) {
            Vec& user = users[i];
            double mind = user.euclideanDistance(centroids[0]);
            int mi = 0;
            for (int c = 1; c < (int)centroids.size(); c++) {
                double cur = user.euclideanDistance(centroids[c]);
                if (cur < mind) { mind = cur; mi = c; }
            }
            ucl[i] = mi;
            std::vector<Vec*> neighbors = clusters[mi];
            if (neighbors.empty()) continue;
            std::vector<int> t = get_top_N_recom(neighbors, user, NTB);
            for (int j = 0; j < NTB; j++) top[(size_t)i * NTB + j] = t[j];
        }
        std::vector<int32_t> nit(1, it);
        write_npy(dir + "/B_rows.npy", rows, {rows.size()});
        write_npy(dir + "/B_assign.npy", assign, {(size_t)F});
        write_npy(dir + "/B_iters.npy", nit, {1});
        write_npy(dir + "/B_centers.npy", centers_of(centroids), {(size_t)K, (size_t)d});
        write_npy(dir + "/B_ucl.npy", ucl, {(size_t)N});
        write_npy(dir + "/B_top.npy", top, {(size_t)N, (size_t)NTB});
        for (auto c : centroids) if (c->getId() == "k_means_center") delete c;
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: ref_harness {lsh|cube|lloyd|kmeanspp|bench} ...\n"); return 2; }
    if (std::string(argv[1]) == "crec") return mode_crec(argc - 1, argv + 1);
    std::string m = argv[1];
    if (m == "lsh") return mode_lsh(argc - 1, argv + 1);
    if (m == "cube") return mode_cube(argc - 1, argv + 1);
    if (m == "lloyd") return mode_lloyd(argc - 1, argv + 1);
    if (m == "kmeanspp") return mode_kmeanspp(argc - 1, argv + 1);
    if (m == "bench") return mode_bench(argc - 1, argv + 1);
    if (m == "recom") return mode_recom(argc - 1, argv + 1);
    if (m == "range") return mode_range(argc - 1, argv + 1);
    if (m == "csv") return mode_csv(argc - 1, argv + 1);
    if (m == "conf") return mode_conf(argc - 1, argv + 1);
    if (m == "c1") return mode_c1(argc - 1, argv + 1);
    if (m == "chain") return mode_chain(argc - 1, argv + 1);
    fprintf(stderr, "unknown mode %s\n", m.c_str());
    return 2;
}
