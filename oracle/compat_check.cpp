// compat_check.cpp — runs the REFERENCE's own functions and the C++ drop-in
// (include/lshkm_compat.hpp, GPU-backed) side by side on the same data and
// seed, through the reference's own interface, and compares everything the
// caller can observe. TEST INFRASTRUCTURE ONLY (tests/test_compat.py).
//
// Built by oracle/Makefile into oracle/_ref/ (git-ignored) from this file, the
// reference's headers/sources where they lie and liblshkm.so; g++ -O0 as the
// reference ships. The reference's clock seed is interposed as in
// ref_harness.cpp so both sides draw from the same engine seed.
//
// usage: compat_check SEED N d K [f64]  -> prints "compat ok" and exits 0, or
// the first mismatches and exits 1. "f64": the components are general doubles
// (not fp32 values; the shim then takes the `_f64` entry points).

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <random>
#include <set>
#include <string>
#include <vector>

static long long g_seed = 1;

namespace std { namespace chrono { inline namespace _V2 {
system_clock::time_point system_clock::now() noexcept {
    return system_clock::time_point(system_clock::duration(g_seed));
}
}}}

#include "utils.hpp"
#include "lsh_cube.hpp"
#include "clustering_phases/assignment.hpp"
#include "clustering_phases/update.hpp"
#include "clustering_phases/initialization.hpp"
#include "crypto_rec.hpp"

#include "../include/lshkm_compat.hpp"
#include "../include/lshkm_synth.h"

typedef CustVector<double> Vec;

static int g_bad = 0;
static bool g_f64 = false;         // the components are general doubles
static bool g_certified = false;   // the shim runs in LSHKM_DIST_CERTIFIED mode
static std::map<std::string, long> g_stat;   // coverage: how much each check exercised
static void fail(const std::string& what) {
    if (g_bad++ < 20) std::printf("MISMATCH %s\n", what.c_str());
}

static std::vector<Vec> make_data(uint64_t seed, int N, int d, bool f64) {
    std::vector<Vec> v;
    v.reserve(N);
    for (int i = 0; i < N; i++) {
        std::vector<double> x(d);
        for (int j = 0; j < d; j++) {
            x[j] = (double)lshkm_synth_value(seed, i, d, j);
            if (f64) x[j] = x[j] * (1.0 + 1e-3 * std::sin(1.0 + 0.7 * j + 1.3 * i)) + 1e-4 * std::cos(j + 0.5 * i);
        }
        v.emplace_back("item" + std::to_string(i), x);
    }
    return v;
}

// queries: dataset rows (alias IDs), perturbed copies under new IDs
static std::vector<Vec> make_queries(std::vector<Vec>& data, int nq) {
    std::vector<Vec> q;
    const int N = (int)data.size();
    for (int i = 0; i < nq; i++) {
        std::vector<double> x = *data[(i * 7919) % N].getDimensions();
        if (i % 2) {
            for (size_t j = 0; j < x.size(); j += 3) x[j] = (double)(float)(x[j] * 0.96875);
            q.emplace_back("query" + std::to_string(i), x);
        } else {
            q.emplace_back(data[(i * 7919) % N].getId(), x);
        }
    }
    return q;
}

static void cmp_ptrs(const std::vector<Vec*>& a, const std::vector<Vec*>& b, const std::string& what) {
    if (a != b) fail(what + " (sizes " + std::to_string(a.size()) + " vs " + std::to_string(b.size()) + ")");
}

static void check_lsh(std::vector<Vec>& data, const std::string& metric, int k, int L, int div, double w) {
    g_seed += 101;
    std::vector<CustHashtable<double>*> ref = create_LSH_hashtables(data, metric, k, L, div, w);
    std::vector<CustHashtable<double>*> gpu = lshkm_compat::create_LSH_hashtables(data, metric, k, L, div, w);  // same clock seed
    const std::string tag = "lsh/" + metric + " ";
    const int nb = metric == "euclidean" ? (int)(data.size() / div) : 1 << k;
    for (int l = 0; l < L; l++)
        for (int b = 0; b < nb; b++)
            cmp_ptrs(ref[l]->getBucketFromIndex(b), gpu[l]->getBucketFromIndex(b),
                     tag + "table " + std::to_string(l) + " bucket " + std::to_string(b));
    std::vector<Vec> qs = make_queries(data, 24);
    for (size_t i = 0; i < qs.size(); i++) {
        for (int l = 0; l < L; l++)
            if (ref[l]->getHash(&qs[i]) != gpu[l]->getHash(&qs[i])) fail(tag + "getHash query " + std::to_string(i));
        cmp_ptrs(get_LSH_combined_buckets(ref, &qs[i]), get_LSH_combined_buckets(gpu, &qs[i]),
                 tag + "combined query " + std::to_string(i));
        std::vector<Vec*> fr = get_LSH_filtered_combined_buckets(ref, &qs[i]);
        cmp_ptrs(fr, get_LSH_filtered_combined_buckets(gpu, &qs[i]), tag + "filtered query " + std::to_string(i));
        g_stat["lsh_" + metric + "_filtered_rows"] += (long)fr.size();
    }
    for (auto t : ref) delete t;
    for (auto t : gpu) delete t;
}

static void check_cube(std::vector<Vec>& data, const std::string& metric, int k, double w) {
    g_seed += 202;
    CustHashtable<double>* ref = create_hypercube(data, metric, k, w);
    CustHashtable<double>* gpu = lshkm_compat::create_hypercube(data, metric, k, w);
    const std::string tag = "cube/" + metric + " ";
    for (int b = 0; b < (1 << k); b++)
        cmp_ptrs(ref->getBucketFromIndex(b), gpu->getBucketFromIndex(b), tag + "bucket " + std::to_string(b));
    // dataset rows only for the euclidean cube: a new h would draw a coin from
    // the engine create_hypercube left on its stack (lsh_cube.hpp:112-118)
    for (int i = 0; i < 16; i++) {
        Vec* q = &data[(i * 613) % data.size()];
        for (int probes : {1, 2, 5, 12}) {
            std::vector<Vec*> pr = get_hypercube_combined_buckets(*ref, q, probes, k);
            cmp_ptrs(pr, get_hypercube_combined_buckets(*gpu, q, probes, k),
                     tag + "probes " + std::to_string(probes) + " query " + std::to_string(i));
            g_stat["cube_" + metric + "_probe_rows"] += (long)pr.size();
        }
    }
    if (metric == "cosine") {
        std::vector<Vec> qs = make_queries(data, 16);
        for (size_t i = 0; i < qs.size(); i++)
            if (ref->getHash(&qs[i]) != gpu->getHash(&qs[i])) fail(tag + "getHash query " + std::to_string(i));
    }
    delete ref;
    delete gpu;
}

// get_P_closest + get_top_N_recom as main.cpp:160-168 chains them. Pool rows
// carry dyadic known means; users get unknown-index sets. Neighbour lists
// include duplicates of one row (ties) and a zero row (NaN similarities).
static void check_recom(std::vector<Vec>& data, int P) {
    const int N = (int)data.size(), d = (int)data[0].getDimensions()->size();
    std::vector<Vec> pool;
    pool.reserve(N + 8);
    for (int i = 0; i < N; i++) {
        std::set<int> none;
        pool.emplace_back("pool" + std::to_string(i), *data[i].getDimensions(), none, ((i * 37) % 33 - 16) / 16.0);
    }
    for (int k = 0; k < 6; k++) {          // duplicates of row 5 and a zero row
        std::set<int> none;
        std::vector<double> v = k < 5 ? *data[5].getDimensions() : std::vector<double>(d, 0.0);
        pool.emplace_back("dup" + std::to_string(k), v, none, 0.25 * k);
    }
    const std::string tag = "recom ";
    for (int q = 0; q < 40; q++) {
        std::set<int> unk;
        for (int j = 0; j < d; j++)
            if ((j * 7 + q * 3) % 5 == 0) unk.insert(j);
        Vec ua("user" + std::to_string(q), *data[(q * 131) % N].getDimensions(), unk, ((q * 11) % 17 - 8) / 8.0);
        Vec ub = ua;
        std::vector<Vec*> na, nb;
        const int n = (q * 53) % (3 * P + 5);
        for (int i = 0; i < n; i++) {
            Vec* p = &pool[(i * 97 + q) % pool.size()];
            na.push_back(p);
        }
        if (q % 4 == 0)
            for (int k = 0; k < 6; k++) na.push_back(&pool[N + k]);
        nb = na;
        if (na.empty()) continue;
        std::vector<double> sa = get_P_closest(na, ua, P);
        std::vector<double> sb = lshkm_compat::get_P_closest(nb, ub, P);
        cmp_ptrs(na, nb, tag + "P-closest order, user " + std::to_string(q));
        if (sa.size() != sb.size() || (!sa.empty() && std::memcmp(sa.data(), sb.data(), sa.size() * sizeof(double))))
            fail(tag + "similarities, user " + std::to_string(q));
        if (get_top_N_recom(na, ua, 5, sa) != lshkm_compat::get_top_N_recom(nb, ub, 5, sb))
            fail(tag + "top-N, user " + std::to_string(q));
        g_stat["recom_users"]++;
    }
}

// main.cpp:149-176 (Part A) as written: cosine LSH over the user vectors, then
// per user get_LSH_filtered_combined_buckets, get_P_closest, get_top_N_recom.
static void check_chain(std::vector<Vec>& data, int k, int L, int P) {
    g_seed += 404;
    std::vector<Vec> users;
    users.reserve(data.size());
    for (size_t i = 0; i < data.size(); i++) {
        std::set<int> unk;
        const int d = (int)data[i].getDimensions()->size();
        for (int j = 0; j < d; j++)
            if ((j * 5 + (int)i) % 7 == 0) unk.insert(j);
        users.emplace_back("u" + std::to_string(i), *data[i].getDimensions(), unk, ((int)(i % 9) - 4) / 8.0);
    }
    std::vector<CustHashtable<double>*> ref = create_LSH_hashtables<double>(users, "cosine", k, L, 100, 0.4);
    std::vector<CustHashtable<double>*> gpu = lshkm_compat::create_LSH_hashtables<double>(users, "cosine", k, L, 100, 0.4);
    const std::string tag = "chain ";
    for (size_t q = 0; q < users.size(); q += 3) {
        Vec& user = users[q];
        std::vector<Vec*> na = get_LSH_filtered_combined_buckets(ref, &user);
        std::vector<Vec*> nb = get_LSH_filtered_combined_buckets(gpu, &user);
        cmp_ptrs(na, nb, tag + "neighbours, user " + std::to_string(q));
        if (na.empty() || na != nb) continue;
        std::vector<double> sa = get_P_closest(na, user, P);
        std::vector<double> sb = lshkm_compat::get_P_closest(nb, user, P);
        cmp_ptrs(na, nb, tag + "P-closest order, user " + std::to_string(q));
        for (size_t i = 0; i < sa.size() && i < sb.size(); i++)
            if (std::memcmp(&sa[i], &sb[i], sizeof(double))) fail(tag + "similarity, user " + std::to_string(q));
        if (sa.size() != sb.size()) fail(tag + "similarity count, user " + std::to_string(q));
        if (get_top_N_recom(na, user, 5, sa) != lshkm_compat::get_top_N_recom(nb, user, 5, sb))
            fail(tag + "top-N, user " + std::to_string(q));
        g_stat["chain_users"]++;
    }
    for (auto t : ref) delete t;
    for (auto t : gpu) delete t;
}

// main.cpp:240-269 (the clustering recommender, Part A): users clustered by the
// reference's own lloyds_assignment, then get_top_N_recom(neighbors, user, 5) --
// the 3-argument overload -- over each user's whole cluster; plus the
// reference's function on an empty list (0/0 predictions) and N past the count.
static void check_cluster_recom(std::vector<Vec>& data, int K) {
    std::vector<Vec> users;
    users.reserve(data.size());
    for (size_t i = 0; i < data.size(); i++) {
        std::set<int> unk;
        const int d = (int)data[i].getDimensions()->size();
        for (int j = 0; j < d; j++)
            if ((j * 3 + (int)i) % 5 == 0) unk.insert(j);
        users.emplace_back("c" + std::to_string(i), *data[i].getDimensions(), unk, ((int)(i % 13) - 6) / 4.0);
    }
    users[3] = Vec("zero", std::vector<double>(data[0].getDimensions()->size(), 0.0), std::set<int>{1, 2}, 0.5);
    const int N = (int)users.size();
    std::vector<Vec*> cents;
    for (int c = 0; c < K; c++) cents.push_back(&users[(size_t)c * (N / K)]);
    lloyds_assignment(users, cents, std::string("euclidean"));
    std::vector<std::vector<Vec*>> clusters = separate_clusters_from_input(users, K);
    const std::string tag = "cluster recom ";
    for (int q = 0; q < N; q += 5) {
        std::vector<Vec*> na = clusters[users[q].getCluster()], nb = na;
        const int nt = q % 3 == 0 ? 5 : (q % 3 == 1 ? 2 : 40);      // 40: past the unknown count (0-padded)
        if (get_top_N_recom(na, users[q], nt) != lshkm_compat::get_top_N_recom(nb, users[q], nt))
            fail(tag + "top-N, user " + std::to_string(q));
        g_stat["cluster_recom_users"]++;
    }
    // main.cpp:260-269 shaped: every user once through the shim, each call with
    // a fresh copy of its cluster (the shim's cluster cache uploads a cluster
    // once, later calls compare it); timed per user
    const auto t0 = std::chrono::steady_clock::now();
    for (int q = 0; q < N; q++) {
        std::vector<Vec*> nb = clusters[users[q].getCluster()];
        (void)lshkm_compat::get_top_N_recom(nb, users[q], 5);
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    g_stat["cluster_recom_shim_us_per_user"] = (long)(us / N + 0.5);
    g_stat["cluster_recom_cache_hits"] = (long)lshkm_compat::cluster_cache().hits;
    // a member changed in place: its cluster's cached copy must not be used
    {
        const int q = 7, c = users[q].getCluster();
        std::vector<double>& x = *clusters[c][0]->getDimensions();
        const double keep = x[0];
        x[0] = keep * 3.0 + 1.0;
        std::vector<Vec*> na = clusters[c], nb = na;
        if (get_top_N_recom(na, users[q], 5) != lshkm_compat::get_top_N_recom(nb, users[q], 5))
            fail(tag + "top-N after a member changed");
        x[0] = keep;
        std::vector<Vec*> na2 = clusters[c], nb2 = na2;
        if (get_top_N_recom(na2, users[q], 5) != lshkm_compat::get_top_N_recom(nb2, users[q], 5))
            fail(tag + "top-N after the member was restored");
    }
    std::vector<Vec*> none_a, none_b;
    if (get_top_N_recom(none_a, users[1], 5) != lshkm_compat::get_top_N_recom(none_b, users[1], 5))
        fail(tag + "empty neighbour list");
}

static void check_init(std::vector<Vec>& data, const std::string& metric, int K) {
    g_seed += 303;
    const std::string tag = "init/" + metric + " ";
    if (k_means_pp(data, K, metric) != lshkm_compat::k_means_pp(data, K, metric)) fail(tag + "k_means_pp");
    if (rand_selection(data, K) != lshkm_compat::rand_selection(data, K)) fail(tag + "rand_selection");
    g_stat["init_" + metric + "_calls"]++;
}

static void check_kmeans(std::vector<Vec>& data, const std::string& metric, int K) {
    std::vector<Vec> a = data, b = data;
    std::vector<Vec*> ca, cb;
    const int N = (int)data.size();
    for (int c = 0; c < K; c++) {
        ca.push_back(&a[(size_t)c * (N / K)]);
        cb.push_back(&b[(size_t)c * (N / K)]);
    }
    const std::string tag = "kmeans/" + metric + " ";
    for (int it = 0; it < 4; it++) {
        lloyds_assignment(a, ca, metric);
        lshkm_compat::lloyds_assignment(b, cb, metric);
        // the distance contract of the shim's mode (lshkm.h Conventions):
        //   exact: the reference's fp64 chain with glibc's pow(x, 2), bit for
        //     bit -- after an update (general fp64 centroids) too;
        //   certified (euclidean only; cosine stays exact-order): <= 2^-20
        //     relative, bit for bit at 0 / inf / NaN.
        const double tol = (g_certified && metric == "euclidean") ? std::ldexp(1.0, -20) : 0.0;
        int nd = 0;
        double worst = 0.0;
        for (int i = 0; i < N; i++) {
            if (a[i].getCluster() != b[i].getCluster()) fail(tag + "cluster of row " + std::to_string(i));
            const double da = a[i].getDistFromCentroid(), db = b[i].getDistFromCentroid();
            if (!(da != 0.0 && std::isfinite(da))) {
                if (std::memcmp(&da, &db, sizeof da)) nd++;
                continue;
            }
            const double rel = std::fabs(da - db) / std::fabs(da);
            worst = std::max(worst, rel);
            if (!(rel <= tol)) nd++;
        }
        if (nd)
            fail(tag + std::to_string(nd) + " distances beyond " + std::to_string(tol) + " rel (worst " +
                 std::to_string(worst) + "), iteration " + std::to_string(it));
        if (tol == 0.0) g_stat["kmeans_" + metric + "_bitexact_iterations"]++;
        const bool ra = k_means(a, ca, metric, 1e-9), rb = lshkm_compat::k_means(b, cb, metric, 1e-9);
        if (ra != rb) fail(tag + "k_means return, iteration " + std::to_string(it));
        for (int c = 0; c < K; c++) {
            if (ca[c]->getId() != cb[c]->getId()) fail(tag + "center id " + std::to_string(c));
            if (*ca[c]->getDimensions() != *cb[c]->getDimensions())
                fail(tag + "center " + std::to_string(c) + " iteration " + std::to_string(it));
        }
        g_stat["kmeans_" + metric + "_iterations"]++;
        if (!ra) break;
    }
    for (int c = 0; c < K; c++) {
        if (ca[c]->getId() == "k_means_center") delete ca[c];
        if (cb[c]->getId() == "k_means_center") delete cb[c];
    }
}

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: compat_check SEED N d K [f64] [exact|certified]\n");
        return 2;
    }
    g_seed = std::atoll(argv[1]);
    const int N = std::atoi(argv[2]), d = std::atoi(argv[3]), K = std::atoi(argv[4]);
    for (int i = 5; i < argc; i++) {
        const std::string a = argv[i];
        if (a == "f64") g_f64 = true;
        else if (a == "certified") g_certified = true;
        else if (a != "exact") { std::fprintf(stderr, "unknown option %s\n", argv[i]); return 2; }
    }
    std::vector<Vec> data = make_data((uint64_t)g_seed, N, d, g_f64);
    try {
        // the shim's default is LSHKM_DIST_EXACT; "certified" opts in
        if (g_certified) lshkm_compat::set_distance_mode(LSHKM_DIST_CERTIFIED);
        check_lsh(data, "euclidean", 4, 5, 50, 4.0);
        check_lsh(data, "cosine", 6, 3, 8, 4.0);
        check_cube(data, "euclidean", 8, 2.0);
        check_cube(data, "cosine", 5, 4.0);
        check_kmeans(data, "euclidean", K);
        check_kmeans(data, "cosine", K);
        check_init(data, "euclidean", K);
        check_init(data, "cosine", K);
        check_recom(data, 10);
        check_cluster_recom(data, K);
        check_chain(data, 4, 5, 20);
    } catch (const std::exception& e) {
        std::printf("EXCEPTION %s\n", e.what());
        return 1;
    }
    if (g_bad) {
        std::printf("compat FAILED: %d mismatches\n", g_bad);
        return 1;
    }
    std::printf("compat ok N=%d d=%d K=%d mode=%s", N, d, K, g_certified ? "certified" : "exact");
    for (const auto& e : g_stat) std::printf(" %s=%ld", e.first.c_str(), e.second);
    std::printf("\n");
    return 0;
}
