"""Regenerate the golden fixtures from the REFERENCE's own code.

Runs oracle/_ref/ref_harness (the reference's lsh_cube.hpp / assignment.hpp /
update.hpp / initialization.hpp compiled from /root/reference with g++ -O0,
clock interposed — see oracle/Makefile) on synthetic inputs and stores the
outputs as tests/golden/<case>.npz plus tests/golden/cases.json.

Inputs are NOT stored: they are the synthetic generator of
include/lshkm_synth.h at the (seed, rows, d) recorded in cases.json, except
external fp64 centroids, which are stored.

Only runs in the build container (the reference is absent on the GPU box).
fp64 cases (kind f64_*, chain, c1 with "f64": true) run on general doubles shaped
like the recommender's user vectors (user_vectors below); their inputs ARE
stored (x64 / q64 / pool ... arrays), as fixtures.

Usage: python tests/golden/make_golden.py [--only lsh,cube,lloyd,kmeanspp,range,csv,conf,c1,recom,f64,chain,crec]
(--only regenerates those kinds and keeps the other cases' entries.)
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")

LSH_CASES = [
    # name, N, d, metric, k, L, div, w, seed, data_seed, nqrows, Q
    ("lsh_e", 1000, 128, "euclidean", 4, 5, 10, 0.4, 777, 1, 20, 10),
    ("lsh_e_w4", 1000, 128, "euclidean", 4, 5, 50, 4.0, 778, 2, 25, 10),
    ("lsh_e_odd", 600, 17, "euclidean", 3, 3, 7, 1.0, 31337, 3, 15, 8),
    ("lsh_c", 1000, 128, "cosine", 4, 5, 0, 0.0, 4242, 4, 10, 5),
    ("lsh_c_odd", 500, 17, "cosine", 5, 2, 0, 0.0, 99, 5, 10, 5),
]
CUBE_CASES = [
    # name, N, d, metric, k, w, seed, data_seed, probes, nqrows, Q
    ("cube_e", 1500, 128, "euclidean", 8, 4.0, 1001, 6, "0,1,2,5,8,20,300", 20, 30),
    ("cube_e14", 3000, 128, "euclidean", 14, 2.0, 1002, 7, "1,14,15", 20, 10),
    ("cube_e_odd", 700, 17, "euclidean", 6, 1.5, 1003, 8, "0,1,3,6,64", 15, 20),
    ("cube_c", 1500, 128, "cosine", 10, 0.0, 1004, 9, "0,1,3,10,50", 20, 10),
]
LLOYD_CASES = [
    # name, N, d, K, metric, iters, min_dist, data_seed, init ("rows" | "ext" | csv of rows)
    ("lloyd_e16", 1000, 128, 16, "euclidean", 3, 0.05, 10, "rows"),
    ("lloyd_e256", 2048, 128, 256, "euclidean", 2, 0.05, 11, "rows"),
    ("lloyd_c16", 1000, 128, 16, "cosine", 3, 0.05, 12, "rows"),
    ("lloyd_ext", 1000, 128, 12, "euclidean", 2, 0.05, 13, "ext"),
    ("lloyd_dup", 800, 32, 8, "euclidean", 3, 0.0, 14, "0,7,7,100,200,200,300,400"),
    ("lloyd_conv", 400, 16, 4, "euclidean", 6, 1e9, 15, "rows"),
    # zero rows (every 37th from row 5): NaN cosine distances and silhouettes
    ("lloyd_c_zero", 600, 24, 6, "cosine", 2, 0.05, 16, "rows"),
    ("lloyd_e_zero", 500, 8, 5, "euclidean", 2, 0.05, 17, "rows"),
    # an external center far from the data: an empty cluster (0/0 silhouette)
    ("lloyd_ext_empty", 700, 16, 6, "euclidean", 2, 0.05, 18, "ext_far"),
]
LLOYD_ZERO_EVERY = {"lloyd_c_zero": 37, "lloyd_e_zero": 37}


def lloyd_data(name, dseed, N, d):
    """Inputs of a Lloyd case (tests rebuild them with conftest.lloyd_input)."""
    x = oracle.synth(dseed, N, d)
    z = LLOYD_ZERO_EVERY.get(name, 0)
    if z:
        x[5::z] = 0.0
    return x
KPP_CASES = [
    # name, N, d, K, metric, seed, data_seed, dup   (config 1 plumbing: 1k x d=16, K=8)
    # dup g: row i is synth row i // g (repeated points: zero distances, repeat picks)
    ("kpp_c1", 1000, 16, 8, "cosine", 2024, 16, 1),
    ("kpp_e1", 1000, 16, 8, "euclidean", 2025, 17, 1),
    ("kpp_e128", 3000, 128, 32, "euclidean", 2026, 18, 1),
    ("kpp_e_big", 40000, 8, 12, "euclidean", 2027, 19, 1),
    ("kpp_dup", 2000, 16, 24, "euclidean", 2028, 20, 4),
    ("kpp_c128", 2000, 128, 16, "cosine", 2029, 21, 1),
]
RANGE_CASES = [
    # name, N, d, K, metric, family, k, L, div, w, probes, iters, min_dist, seed, data_seed, dup
    # (dup g: row i is synth row i // g; g > N/K makes centroids 0 and 1 equal: radius 0)
    ("range_lsh_e", 1500, 128, 16, "euclidean", "lsh", 4, 5, 10, 4.0, 0, 3, 0.01, 5001, 30, 1),
    ("range_lsh_c", 1200, 64, 12, "cosine", "lsh", 5, 3, 1, 0.0, 0, 2, 0.01, 5002, 31, 1),
    ("range_lsh_k3", 900, 16, 3, "euclidean", "lsh", 3, 4, 9, 2.0, 0, 3, 0.0, 5003, 32, 1),
    ("range_lsh_dup", 800, 24, 8, "euclidean", "lsh", 3, 3, 8, 2.0, 0, 2, 0.0, 5004, 33, 150),
    ("range_cube_e", 1500, 32, 12, "euclidean", "cube", 6, 1, 1, 2.0, 3, 1, 0.0, 5005, 34, 1),
    ("range_cube_c", 1500, 128, 20, "cosine", "cube", 8, 1, 1, 0.0, 8, 1, 0.0, 5006, 35, 1),
]
# Input-format cases: files written here under tests/golden/io/ (our own data in
# the reference's formats), parsed by the reference's VectorReader / ArgParser.
CSV_CASES = [
    # name, delimiter (ASCII), strt_line, N, d, seed
    ("csv_comma", 44, 1, 400, 16, 6001),
    ("csv_tab_meta", 9, 3, 300, 7, 6002),
    ("csv_space", 32, 2, 200, 33, 6003),
]
# Config C1 (BASELINE.json configs[0]): main.cpp:81-111 on a 1k x 16 CSV, K=8
C1_CASES = [
    # name, N, d, K, iters, min_dist, seed, data_seed
    ("c1_proj2", 1000, 16, 8, 30, 0.05, 7001, 7002),
    ("c1_proj2_b", 1500, 16, 8, 5, 0.0, 7003, 7004),
]
CONF_KEYS = ["proj_2_input", "proj_2_csv_delimiter", "proj_2_number_of_clusters", "number_of_clusters",
             "number_of_hash_functions", "number_of_hash_tables", "csv_delimiter", "lsh_bucket_div", "euclidean_h_w",
             "cube_range_c", "cube_probes", "max_algo_iterations", "min_dist_kmeans", "metric_type", "lexicon_file",
             "query_file", "missing_key", "//", "k"]
CONF_CASES = {
    "conf_a": "// options, one per line\nproj_2_input ./p2.csv\nproj_2_csv_delimiter ,\nproj_2_number_of_clusters 8\n\n"
              "number_of_clusters 12 // k\nnumber_of_hash_functions 3 //default:4\nnumber_of_hash_tables  6\n"
              "csv_delimiter 9 // ASCII CODE\r\nlsh_bucket_div 50\neuclidean_h_w 0.25\nmax_algo_iterations 7\n"
              "min_dist_kmeans 1e-3\nmetric_type euclidean\nlexicon_file lex.csv\nquery_file q.csv",
    "conf_c": "proj_2_input ../in.csv\nproj_2_csv_delimiter ;\nproj_2_number_of_clusters 20\n\nnumber_of_clusters 30 // k\n"
              "number_of_hash_functions 4 //default:4\nnumber_of_hash_tables 5 //default:L=5\n\ncsv_delimiter 44 // ASCII CODE\n\n"
              "lsh_bucket_div 100\neuclidean_h_w 0.4\n\nmax_algo_iterations 1\nmin_dist_kmeans 0.05\n\nmetric_type cosine\n",
    "conf_b": "number_of_clusters 4\nnumber_of_clusters 9\neuclidean_h_w -2.5e+1xyz\nquery_file\n",
}


def csv_text(name, delim, strt, N, d, seed):
    """Numbers in many spellings std::stod accepts: %.17g, short, exponent,
    hex float, signs, leading blanks, inf/nan; \r\n on some lines, a trailing
    delimiter on others."""
    rng = np.random.default_rng(seed)
    D = chr(delim)
    lines = [f"meta line {i} {D} x" for i in range(strt - 1)]
    for i in range(N):
        vals = []
        for j in range(d):
            v = rng.standard_normal() * 10.0 ** int(rng.integers(-6, 7))
            k = int(rng.integers(0, 12))
            if k == 0: t = "%.17g" % v
            elif k == 1: t = "%g" % v
            elif k == 2: t = "%.3e" % v
            elif k == 3: t = float(np.float32(v)).hex()
            elif k == 4: t = "+%d" % int(v) if v >= 0 else "%d" % int(v)
            elif k == 5: t = ("  " if D != " " else "") + repr(float(np.float32(v)))
            elif k == 6: t = "-0"
            elif k == 7 and (i + j) % 97 == 0: t = "inf" if v > 0 else "-INF"
            elif k == 8 and (i + j) % 89 == 0: t = "nan"
            else: t = repr(float(v))
            vals.append(t)
        line = f"u{i:05d}" + D + D.join(vals)
        if i % 7 == 3: line += D
        if i % 5 == 1: line += "\r"
        lines.append(line)
    return "\n".join(lines) + ("\n" if seed % 2 else "")


RECOM_CASES = [
    # name, N, d, Q, P, NTOP, seed, values ("dyadic": k/8, squares exact; "f64": general doubles)
    ("recom_dy", 300, 20, 80, 10, 5, 4001, "dyadic"),
    ("recom_f64", 400, 24, 60, 15, 2, 4002, "f64"),
    ("recom_big", 3000, 16, 12, 40, 5, 4003, "dyadic"),
]


def recom_inputs(N, d, Q, seed, values):
    """Pool rows (with duplicates and a zero row: equal / NaN similarities),
    users (some are pool rows, as in main.cpp's part A), means, unknown index
    sets and ascending candidate lists of every size class (0, 1, P, N)."""
    rng = np.random.default_rng(seed)
    if values == "dyadic":
        X = rng.integers(-40, 41, size=(N, d)).astype(np.float64) / 8.0
        xm = rng.integers(-32, 33, size=N).astype(np.float64) / 16.0
    else:
        X = rng.standard_normal((N, d)) * 1.7
        xm = rng.standard_normal(N)
    for i in range(0, N, 7):                      # duplicates of earlier rows
        X[i] = X[(i * 13) % max(i, 1)]
    X[N // 2] = 0.0                               # zero row: NaN similarities
    X[N // 3] = 2.0 * X[N // 5]                   # parallel rows: equal similarities
    U = X[rng.integers(0, N, size=Q)].copy()
    for q in range(0, Q, 3):
        U[q] = (rng.integers(-40, 41, size=d) / 8.0) if values == "dyadic" else rng.standard_normal(d)
    um = (rng.integers(-32, 33, size=Q) / 16.0) if values == "dyadic" else rng.standard_normal(Q)
    unk, cand = [], []
    sizes = [0, 1, 2, 5, 10, 11, 40, N]
    for q in range(Q):
        m = int(rng.integers(0, d + 1)) if q % 5 else int(rng.integers(0, 3))
        unk.append(np.sort(rng.choice(d, size=m, replace=False)).astype(np.int32))
        n = sizes[q % len(sizes)] if q < 2 * len(sizes) else int(rng.integers(0, N + 1))
        cand.append(np.sort(rng.choice(N, size=n, replace=False)).astype(np.int32))
    csr = lambda ls: (np.cumsum([0] + [len(l) for l in ls]).astype(np.int64),
                      np.concatenate(ls).astype(np.int32) if ls else np.zeros(0, np.int32))
    up, ui = csr(unk)
    cp, ci = csr(cand)
    return dict(x=X, xmean=xm, u=U, umean=um.astype(np.float64), unk_ptr=up, unk_idx=ui, cand_ptr=cp, cand_idx=ci)


def user_vectors(seed, N, d):
    """General doubles shaped like tweets_to_user_vectors (crypto_rec.hpp:78-140):
    per user a few tweets, each mentioning 1-3 coins with a sentiment score
    s = x / sqrt(x^2 + 15) (tweet.cpp) over a lexicon sum x of +-k/4 words;
    positive scores accumulate on the mentioned coins; every unmentioned coin
    gets the mean of the known ones (summed in index order, as the reference).
    Users with an all-zero vector are redrawn (the reference drops them).
    Returns (X [N][d] fp64, unknown index lists, known means)."""
    rng = np.random.RandomState(seed)
    X = np.zeros((N, d))
    unk, means = [], np.zeros(N)
    for i in range(N):
        while True:
            x = np.zeros(d)
            known = np.zeros(d, bool)
            for _ in range(1 + rng.poisson(4)):
                coins = rng.choice(d, size=1 + rng.randint(3), replace=False)
                lex = float(sum(rng.randint(-8, 9) for _ in range(1 + rng.randint(4)))) / 4.0
                sc = lex / np.sqrt(lex * lex + 15.0)
                for c in coins:
                    if sc > 0:
                        x[c] = x[c] + sc
                    known[c] = True
            if (x != 0).any():
                break
        tot, cnt = 0.0, 0
        for j in range(d):
            if known[j]:
                tot = tot + x[j]
                cnt += 1
        mean = tot / cnt
        x[~known] = mean
        X[i] = x
        unk.append(np.nonzero(~known)[0].astype(np.int32))
        means[i] = mean
    return X, unk, means


def csr_of(lists):
    return (np.cumsum([0] + [len(l) for l in lists]).astype(np.int64),
            np.concatenate(lists).astype(np.int32) if lists else np.zeros(0, np.int32))


F64_CASES = [
    # name, kind, N, d, params..., data seed  (rows: user_vectors(seed, N, d); queries: seed + 1)
    ("lsh_e64", "lsh", 700, 100, dict(metric="euclidean", k=4, L=5, div=10, w=0.4, seed=811, nqrows=20, Q=15), 8001),
    ("lsh_c64", "lsh", 700, 100, dict(metric="cosine", k=4, L=5, div=1, w=0.0, seed=812, nqrows=20, Q=15), 8002),
    ("lsh_e64_odd", "lsh", 400, 23, dict(metric="euclidean", k=3, L=3, div=7, w=0.25, seed=813, nqrows=10, Q=10), 8003),
    ("cube_e64", "cube", 900, 100, dict(metric="euclidean", k=8, w=0.5, seed=821, probes="0,1,2,8,30", nqrows=20, Q=15), 8004),
    ("cube_c64", "cube", 900, 100, dict(metric="cosine", k=10, w=0.0, seed=822, probes="0,1,3,10", nqrows=20, Q=15), 8005),
    ("lloyd_e64", "lloyd", 1000, 100, dict(K=16, metric="euclidean", iters=3, min_dist=0.0), 8006),
    ("lloyd_c64", "lloyd", 1000, 100, dict(K=12, metric="cosine", iters=3, min_dist=0.0), 8007),
    ("lloyd_e64_k80", "lloyd", 1200, 40, dict(K=80, metric="euclidean", iters=2, min_dist=0.0), 8008),
    ("kpp_e64", "kmeanspp", 1500, 100, dict(K=16, metric="euclidean", seed=831), 8009),
    ("kpp_c64", "kmeanspp", 1500, 100, dict(K=16, metric="cosine", seed=832), 8010),
    ("range_lsh_e64", "range", 900, 100, dict(K=12, metric="euclidean", family="lsh", k=4, L=5, div=10, w=1.0,
                                             probes=0, iters=2, min_dist=0.0, seed=841), 8011),
    ("range_cube_c64", "range", 900, 100, dict(K=12, metric="cosine", family="cube", k=8, L=1, div=1, w=0.0,
                                              probes=6, iters=1, min_dist=0.0, seed=842), 8012),
]
# main.cpp's cosine LSH recommender, Part A (users indexed and queried) and Part B
# (tables over another pool, queried with the users): name, N, Q, d, k, L, w, seed, P, NTOP, self, data seed
CHAIN_CASES = [
    ("chain_a", 600, 600, 100, 4, 5, 0.4, 851, 20, 5, 1, 8101),
    ("chain_b", 500, 300, 100, 4, 5, 0.4, 852, 20, 2, 0, 8102),
    ("chain_a_k6", 400, 400, 60, 6, 3, 0.4, 853, 10, 5, 1, 8103),
]

# main.cpp's clustering recommenders (Part A: rand_selection + Lloyd/k_means on the
# user vectors, each user's own cluster; Part B: k_means_pp + Lloyd/k_means on
# the "fake" user vectors, each user's nearest centroid), both with the
# 3-argument get_top_N_recom (crypto_rec.hpp:327-345):
# name, N users, F fake users, d, K, iters, min_dist, seedA, seedB, NTA, NTB, data seed, fake dup
# (fake dup g: each distinct fake user appears g times in a row -- more
# centroids than distinct points: k_means_pp's all-zero minima, duplicate
# centroids, empty clusters)
CREC_CASES = [
    ("crec_a", 600, 500, 100, 12, 5, 0.0, 861, 862, 5, 2, 8201, 1),
    ("crec_b", 300, 60, 60, 30, 4, 0.0, 863, 864, 5, 2, 8202, 3),      # 20 distinct fake users, K = 30
    ("crec_c", 500, 400, 24, 8, 30, 0.05, 865, 866, 7, 3, 8203, 1),    # converges before the iteration cap
    # user vectors scaled per user by 16 exp(U(-0.3, 0.3)) and rounded to 2^-24
    # (25-28 significant bits): many squares are exact ties, which glibc's
    # pow(x, 2) rounds unlike x*x, so the norms differ on >= 1 % of the users
    # (checked below; plain general doubles absorb the last-bit differences of
    # their squares in the sums almost always)
    ("crec_pw", 1000, 600, 100, 16, 4, 0.0, 867, 868, 5, 3, 8204, 1),
]
CREC_GENERAL = {"crec_pw"}


def pow_norm_disagreement(X):
    """Fraction of rows whose sequential sum of pow(x, 2) differs from the sum of x*x."""
    import math
    n = 0
    for x in X:
        a = b = 0.0
        for v in x:
            a = a + math.pow(float(v), 2)
            b = b + float(v) * float(v)
        n += a != b
    return n / max(len(X), 1)


def run(args):
    subprocess.run([HARNESS] + [str(a) for a in args], check=True)


def load_dir(d):
    return {f[:-4]: np.load(os.path.join(d, f)) for f in sorted(os.listdir(d)) if f.endswith(".npy")}


def ext_centers(seed, K, d):
    # Deterministic non-fp32 fp64 centers: synth rows scaled by (1 + small irrational offsets).
    base = oracle.synth(seed, K, d).astype(np.float64)
    j = np.arange(d, dtype=np.float64)[None, :]
    c = np.arange(K, dtype=np.float64)[:, None]
    return base * (1.0 + 1e-3 * np.sin(1.0 + j * 0.7 + c * 1.3)) + 1e-4 * np.cos(j + c)


def kpp_data(dseed, N, d, dup):
    """Inputs of a k-means++ case (tests rebuild them the same way)."""
    return oracle.synth(dseed, N, d)[np.arange(N) // dup]


def main(only=None):
    if not os.path.exists(HARNESS):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    meta = {}
    if only:
        with open(os.path.join(HERE, "cases.json")) as f:
            meta = {k: v for k, v in json.load(f).items() if v["kind"] not in only}
    want = (lambda kind: only is None or kind in only)
    tmp = tempfile.mkdtemp()
    try:
        for (name, N, d, metric, k, L, div, w, seed, dseed, nqrows, Q) in (LSH_CASES if want("lsh") else []):
            out = os.path.join(tmp, name); os.makedirs(out)
            x = oracle.synth(dseed, N, d); x.tofile(os.path.join(tmp, "x.f32"))
            q = oracle.synth(dseed + 1000, Q, d); q.tofile(os.path.join(tmp, "q.f32"))
            run(["lsh", os.path.join(tmp, "x.f32"), N, d, metric, k, L, div if div else 1, w, seed, out,
                 os.path.join(tmp, "q.f32"), Q, nqrows])
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **load_dir(out))
            meta[name] = dict(kind="lsh", N=N, d=d, metric=metric, k=k, L=L, div=div, w=w, seed=seed,
                              data_seed=dseed, query_seed=dseed + 1000, nqrows=nqrows, Q=Q,
                              nb=(N // div) if metric == "euclidean" else 2 ** k)
        for (name, N, d, metric, k, w, seed, dseed, probes, nqrows, Q) in (CUBE_CASES if want("cube") else []):
            out = os.path.join(tmp, name); os.makedirs(out)
            x = oracle.synth(dseed, N, d); x.tofile(os.path.join(tmp, "x.f32"))
            q = oracle.synth(dseed + 1000, Q, d); q.tofile(os.path.join(tmp, "q.f32"))
            run(["cube", os.path.join(tmp, "x.f32"), N, d, metric, k, w, seed, probes, out,
                 os.path.join(tmp, "q.f32"), Q, nqrows])
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **load_dir(out))
            meta[name] = dict(kind="cube", N=N, d=d, metric=metric, k=k, w=w, seed=seed, data_seed=dseed,
                              query_seed=dseed + 1000, probes=[int(p) for p in probes.split(",")],
                              nqrows=nqrows, Q=Q)
        for (name, N, d, K, metric, iters, min_dist, dseed, init) in (LLOYD_CASES if want("lloyd") else []):
            out = os.path.join(tmp, name); os.makedirs(out)
            x = lloyd_data(name, dseed, N, d); x.tofile(os.path.join(tmp, "x.f32"))
            args = ["lloyd", os.path.join(tmp, "x.f32"), N, d, K, metric, iters, repr(min_dist), out]
            extra = {}
            if init in ("ext", "ext_far"):
                c = ext_centers(dseed + 500, K, d)
                if init == "ext_far":
                    c[K // 2] += 1e3
                c.tofile(os.path.join(tmp, "c.f64"))
                args += [os.path.join(tmp, "c.f64")]
                extra["ext_centers"] = c
            elif init != "rows":
                args += ["-", init]
            run(args)
            res = load_dir(out); res.update(extra)
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
            meta[name] = dict(kind="lloyd", N=N, d=d, K=K, metric=metric, iters=iters, min_dist=min_dist,
                              data_seed=dseed, init=init, zero_every=LLOYD_ZERO_EVERY.get(name, 0))
        for (name, N, d, K, metric, seed, dseed, dup) in (KPP_CASES if want("kmeanspp") else []):
            out = os.path.join(tmp, name); os.makedirs(out)
            x = kpp_data(dseed, N, d, dup); x.tofile(os.path.join(tmp, "x.f32"))
            run(["kmeanspp", os.path.join(tmp, "x.f32"), N, d, K, metric, seed, out])
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **load_dir(out))
            meta[name] = dict(kind="kmeanspp", N=N, d=d, K=K, metric=metric, seed=seed, data_seed=dseed, dup=dup)
        for (name, N, d, K, metric, fam, k, L, div, w, probes, iters, md, seed, dseed, dup) in \
                (RANGE_CASES if want("range") else []):
            out = os.path.join(tmp, name); os.makedirs(out)
            x = kpp_data(dseed, N, d, dup); x.tofile(os.path.join(tmp, "x.f32"))
            run(["range", os.path.join(tmp, "x.f32"), N, d, K, metric, fam, k, L, div, w, probes, iters,
                 repr(md), seed, out])
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **load_dir(out))
            meta[name] = dict(kind="range", N=N, d=d, K=K, metric=metric, family=fam, k=k, L=L, div=div, w=w,
                              probes=probes, iters=iters, min_dist=md, seed=seed, data_seed=dseed, dup=dup)
        iodir = os.path.join(HERE, "io")
        if want("csv") or want("conf"):
            os.makedirs(iodir, exist_ok=True)
        for (name, delim, strt, N, d, seed) in (CSV_CASES if want("csv") else []):
            path = os.path.join(iodir, name + ".csv")
            with open(path, "w", newline="") as f:
                f.write(csv_text(name, delim, strt, N, d, seed))
            out = os.path.join(tmp, name); os.makedirs(out)
            run(["csv", path, delim, strt, out])
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **load_dir(out))
            meta[name] = dict(kind="csv", delim=delim, strt_line=strt, N=N, d=d, file="io/" + name + ".csv")
        if want("c1") or want("csv") or want("conf"):
            os.makedirs(iodir, exist_ok=True)
        for (name, N, d, K, iters, md, seed, dseed) in (C1_CASES if want("c1") else []):
            x = oracle.synth(dseed, N, d)
            path = os.path.join(iodir, name + ".csv")
            with open(path, "w") as f:
                for i in range(N):
                    f.write(f"{i}," + ",".join(repr(float(v)) for v in x[i]) + "\n")
            out = os.path.join(tmp, name); os.makedirs(out)
            run(["c1", path, 44, K, iters, repr(md), seed, out])
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **load_dir(out))
            meta[name] = dict(kind="c1", N=N, d=d, K=K, iters=iters, min_dist=md, seed=seed, data_seed=dseed,
                              file="io/" + name + ".csv")
        # config C1 on an unquantized CSV: general doubles written with %.17g
        for (name, N, d, K, iters, md, seed, dseed) in ([("c1_proj2_f64", 1000, 16, 8, 30, 0.05, 7005, 7006)]
                                                       if want("c1") else []):
            rng = np.random.RandomState(dseed)
            x = rng.standard_normal((N, d)) * np.exp(rng.uniform(-2, 2, size=(N, 1)))
            path = os.path.join(iodir, name + ".csv")
            with open(path, "w") as f:
                for i in range(N):
                    f.write(f"{i}," + ",".join("%.17g" % float(v) for v in x[i]) + "\n")
            out = os.path.join(tmp, name); os.makedirs(out)
            run(["c1", path, 44, K, iters, repr(md), seed, out])
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **load_dir(out))
            meta[name] = dict(kind="c1", N=N, d=d, K=K, iters=iters, min_dist=md, seed=seed, data_seed=dseed,
                              file="io/" + name + ".csv", f64=True)
        for (name, kind, N, d, pr, dseed) in (F64_CASES if want("f64") else []):
            out = os.path.join(tmp, name); os.makedirs(out)
            x, _, _ = user_vectors(dseed, N, d)
            xf = os.path.join(tmp, "x.f64"); x.tofile(xf)
            stored = dict(x64=x)
            if kind == "lsh":
                q, _, _ = user_vectors(dseed + 1, pr["Q"], d); qf = os.path.join(tmp, "q.f64"); q.tofile(qf)
                stored["q64"] = q
                run(["lsh", xf, N, d, pr["metric"], pr["k"], pr["L"], pr["div"], pr["w"], pr["seed"], out, qf,
                     pr["Q"], pr["nqrows"]])
                pr = dict(pr, nb=(N // pr["div"]) if pr["metric"] == "euclidean" else 2 ** pr["k"])
            elif kind == "cube":
                q, _, _ = user_vectors(dseed + 1, pr["Q"], d); qf = os.path.join(tmp, "q.f64"); q.tofile(qf)
                stored["q64"] = q
                run(["cube", xf, N, d, pr["metric"], pr["k"], pr["w"], pr["seed"], pr["probes"], out, qf, pr["Q"],
                     pr["nqrows"]])
                pr = dict(pr, probes=[int(v) for v in pr["probes"].split(",")])
            elif kind == "lloyd":
                run(["lloyd", xf, N, d, pr["K"], pr["metric"], pr["iters"], repr(pr["min_dist"]), out])
            elif kind == "kmeanspp":
                run(["kmeanspp", xf, N, d, pr["K"], pr["metric"], pr["seed"], out])
            elif kind == "range":
                run(["range", xf, N, d, pr["K"], pr["metric"], pr["family"], pr["k"], pr["L"], pr["div"], pr["w"],
                     pr["probes"], pr["iters"], repr(pr["min_dist"]), pr["seed"], out])
            res = load_dir(out); res.update(stored)
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
            meta[name] = dict(kind="f64_" + kind, N=N, d=d, data_seed=dseed, **pr)
        for (name, N, Q, d, k, L, w, seed, P, NT, self_, dseed) in (CHAIN_CASES if want("chain") else []):
            out = os.path.join(tmp, name); os.makedirs(out)
            pool, punk, pmean = user_vectors(dseed, N, d)
            inp = dict(pool=pool, pmean=pmean)
            inp["punk_ptr"], inp["punk_idx"] = csr_of(punk)
            if not self_:
                users, uunk, umean = user_vectors(dseed + 1, Q, d)
                inp.update(users=users, umean=umean)
                inp["uunk_ptr"], inp["uunk_idx"] = csr_of(uunk)
            ext = dict(pool="f64", pmean="f64", punk_ptr="i64", punk_idx="i32", users="f64", umean="f64",
                       uunk_ptr="i64", uunk_idx="i32")
            for kk, v in inp.items():
                v.tofile(os.path.join(out, f"{kk}.{ext[kk]}"))
            run(["chain", out, N, Q, d, k, L, 1, w, seed, P, NT, self_])
            res = load_dir(out); res.update(inp)
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
            meta[name] = dict(kind="chain", N=N, Q=N if self_ else Q, d=d, k=k, L=L, w=w, seed=seed, P=P, NTOP=NT,
                              self=bool(self_), data_seed=dseed)
        for (name, N, F, d, K, iters, md, sa, sb, nta, ntb, dseed, dup) in (CREC_CASES if want("crec") else []):
            out = os.path.join(tmp, name); os.makedirs(out)
            users, uunk, umean = user_vectors(dseed, N, d)
            fake, funk, fmean = user_vectors(dseed + 1, F // dup, d)
            if name in CREC_GENERAL:
                rs = np.random.RandomState(dseed + 2)
                su, sf = 16.0 * np.exp(rs.uniform(-0.3, 0.3, N)), 16.0 * np.exp(rs.uniform(-0.3, 0.3, len(fake)))
                q = lambda v: np.round(v * 2.0 ** 24) / 2.0 ** 24
                users, umean = q(users * su[:, None]), q(umean * su)
                fake, fmean = q(fake * sf[:, None]), q(fmean * sf)
                fr = pow_norm_disagreement(users)
                assert fr >= 0.01, fr
                print(f"{name}: pow(x, 2) vs x*x differ on {100 * fr:.1f} % of the user norms")
            fake, fmean = np.repeat(fake, dup, axis=0), np.repeat(fmean, dup)
            funk = [u for u in funk for _ in range(dup)]
            inp = dict(users=users, umean=umean, fake=fake, fmean=fmean)
            inp["uunk_ptr"], inp["uunk_idx"] = csr_of(uunk)
            inp["funk_ptr"], inp["funk_idx"] = csr_of(funk)
            ext = dict(users="f64", umean="f64", fake="f64", fmean="f64", uunk_ptr="i64", uunk_idx="i32",
                       funk_ptr="i64", funk_idx="i32")
            for kk, v in inp.items():
                v.tofile(os.path.join(out, f"{kk}.{ext[kk]}"))
            run(["crec", out, N, F, d, K, iters, repr(md), sa, sb, nta, ntb])
            res = load_dir(out); res.update(inp)
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
            meta[name] = dict(kind="crec", N=N, F=F, d=d, K=K, iters=iters, min_dist=md, seedA=sa, seedB=sb,
                              NTA=nta, NTB=ntb, data_seed=dseed, fake_dup=dup)
        for name, text in (CONF_CASES.items() if want("conf") else []):
            path = os.path.join(iodir, name + ".conf")
            with open(path, "w", newline="") as f:
                f.write(text)
            res = subprocess.run([HARNESS, "conf", path] + CONF_KEYS, check=True, capture_output=True, text=True)
            vals = {}
            for key, ln in zip(CONF_KEYS, res.stdout.split("\n")):
                vals[key] = ln[2:] if ln.startswith("1 ") else None
            meta[name] = dict(kind="conf", file="io/" + name + ".conf", values=vals)
        for (name, N, d, Q, P, NT, seed, values) in (RECOM_CASES if want("recom") else []):
            out = os.path.join(tmp, name); os.makedirs(out)
            inp = recom_inputs(N, d, Q, seed, values)
            ext = dict(x="f64", xmean="f64", u="f64", umean="f64", unk_ptr="i64", unk_idx="i32",
                       cand_ptr="i64", cand_idx="i32")
            for k, e in ext.items():
                inp[k].tofile(os.path.join(out, f"{k}.{e}"))
            run(["recom", out, N, d, Q, P, NT])
            res = load_dir(out); res.update(inp)
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **res)
            meta[name] = dict(kind="recom", N=N, d=d, Q=Q, P=P, NTOP=NT, seed=seed, values=values)
    finally:
        shutil.rmtree(tmp)
    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    total = sum(os.path.getsize(os.path.join(HERE, n + ".npz")) for n in meta if os.path.exists(os.path.join(HERE, n + ".npz")))
    print(f"wrote {len(meta)} cases, {total / 1e6:.2f} MB")


if __name__ == "__main__":
    only = None
    if len(sys.argv) > 2 and sys.argv[1] == "--only":
        only = set(sys.argv[2].split(","))
    main(only)
