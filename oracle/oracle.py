"""ctypes front-end of the CPU oracle (oracle/_ref/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker (or the timed CPU
baseline), never as the product. The product package never imports this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
u32ref = C.POINTER(C.c_uint32)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_ref", "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        sig = {
            "or_minstd_seed": (C.c_uint32, [C.c_uint64]),
            "or_uniform_int": (C.c_int, [u32ref, C.c_int, C.c_int]),
            "or_gen_lsh_euclid": (C.c_uint32, [C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_float, f32p, f32p, i32p]),
            "or_gen_lsh_cosine": (C.c_uint32, [C.c_uint64, C.c_int, C.c_int, C.c_int, f64p]),
            "or_gen_cube_euclid": (C.c_uint32, [C.c_uint64, C.c_int, C.c_int, C.c_float, f32p, f32p]),
            "or_gen_cube_cosine": (C.c_uint32, [C.c_uint64, C.c_int, C.c_int, f64p]),
            "or_lsh_hash_euclid": (None, [C.c_int64, C.c_int, C.c_int, C.c_int, f64p, f32p, f32p, C.c_float,
                                          i32p, C.c_int64, i32p, i32p, i32p]),
            "or_lsh_hash_cosine": (None, [C.c_int64, C.c_int, C.c_int, C.c_int, f64p, f64p, i32p]),
            "or_bucket_csr": (None, [C.c_int64, C.c_int, C.c_int64, i32p, i64p, i32p]),
            "or_lsh_query": (C.c_int64, [C.c_int64, C.c_int, C.c_int, C.c_int64, C.c_void_p, i64p, i32p,
                                         C.c_void_p, i32p, i32p, C.c_int64]),
            "or_cube_h": (None, [C.c_int64, C.c_int, C.c_int, f64p, f32p, f32p, C.c_float, i32p]),
            "or_cube_coins": (C.c_int64, [C.c_int64, C.c_int, i32p, C.c_int32, C.c_int32, i32p, u32ref, i32p]),
            "or_cube_cosine": (None, [C.c_int64, C.c_int, C.c_int, f64p, f64p, i32p]),
            "or_cube_probe_seq": (C.c_int64, [C.c_int32, C.c_int, C.c_int, i32p, C.c_int64]),
            "or_lloyd_assign": (None, [C.c_int64, C.c_int, C.c_int, f64p, f64p, C.c_int, C.c_void_p, i32p, f64p]),
            "or_kmeans_update": (C.c_int, [C.c_int64, C.c_int, C.c_int, f64p, i32p, f64p, C.c_int, C.c_double,
                                           f64p, i64p]),
            "or_range_assign": (C.c_int, [C.c_int64, C.c_int, C.c_int, f64p, f64p, C.c_int, i64p, i32p,
                                          C.c_void_p, C.c_void_p, i32p, f64p]),
            "or_silhouette": (None, [C.c_int64, C.c_int, C.c_int, f64p, i32p, f64p, C.c_int, f64p, C.c_void_p]),
            "or_rand_selection": (None, [C.c_uint64, C.c_int64, C.c_int, i32p]),
            "or_kmeans_pp": (None, [C.c_int64, C.c_int, C.c_int, f64p, C.c_int, C.c_uint64, i32p]),
            "or_p_closest": (None, [C.c_int, f64p, C.c_int64, f64p, i64p, i32p, C.c_int, i32p, f64p, i32p]),
            "or_top_n_recom": (None, [C.c_int, f64p, f64p, C.c_int64, f64p, f64p, i64p, i32p, i32p, f64p, i32p,
                                      C.c_int, C.c_int, i32p]),
            "or_cluster_top_n": (None, [C.c_int, f64p, f64p, i64p, i32p, C.c_int64, f64p, f64p, i32p, i64p, i32p,
                                        C.c_int, i32p]),
            "or_synth": (None, [C.c_uint64, C.c_int64, C.c_int64, C.c_int, f32p]),
            "or_synth_normal": (None, [C.c_uint64, C.c_int64, C.c_int64, C.c_int, f32p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def rows64(X):
    """Dataset rows as the reference holds them (fp64; fp32 data widens exactly)."""
    return np.ascontiguousarray(X, np.float64)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def synth(seed, rows, d, row0=0, kind="grid"):
    """include/lshkm_synth.h: kind "grid" (Irwin-Hall(4) on a 2^-15 grid) or
    "normal" (Irwin-Hall(12), full fp32 mantissas)."""
    out = np.empty((rows, d), np.float32)
    (lib().or_synth_normal if kind == "normal" else lib().or_synth)(seed, row0, rows, d, out)
    return out


def synth_normal_np(seed, rows, d, row0=0):
    """The "normal" generator restated in numpy (uint64 arithmetic), a second
    producer of the same bits."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        e = (np.arange(rows, dtype=np.uint64)[:, None] + np.uint64(row0)) * np.uint64(d) + np.arange(d, dtype=np.uint64)
        base = np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + e * np.uint64(12)
        s = np.full(base.shape, -(6 << 40), np.int64)
        for k in range(12):
            x = base + np.uint64(k) + np.uint64(0x9E3779B97F4A7C15)
            x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            x = x ^ (x >> np.uint64(31))
            s += (x >> np.uint64(24)).astype(np.int64)
    del M
    return (s.astype(np.float32) * np.float32(2.0 ** -40)).astype(np.float32)


def gen_lsh_euclid(seed, L, k, d, w):
    V = np.empty((L, k, d), np.float32); t = np.empty((L, k), np.float32); r = np.empty((L, k), np.int32)
    st = lib().or_gen_lsh_euclid(seed, L, k, d, w, V, t, r)
    return V, t, r, st


def gen_lsh_cosine(seed, L, k, d):
    R = np.empty((L, k, d), np.float64)
    st = lib().or_gen_lsh_cosine(seed, L, k, d, R)
    return R, st


def gen_cube_euclid(seed, k, d, w):
    V = np.empty((k, d), np.float32); t = np.empty((k,), np.float32)
    st = lib().or_gen_cube_euclid(seed, k, d, w, V, t)
    return V, t, st


def gen_cube_cosine(seed, k, d):
    R = np.empty((k, d), np.float64)
    st = lib().or_gen_cube_cosine(seed, k, d, R)
    return R, st


def lsh_hash_euclid(X, V, t, w, r, nb):
    X = rows64(X)
    N, d = X.shape; L, k = t.shape
    tuples = np.empty((N, L, k), np.int32); phi = np.empty((N, L), np.int32); bucket = np.empty((N, L), np.int32)
    lib().or_lsh_hash_euclid(N, d, L, k, X, np.ascontiguousarray(V, np.float32), np.ascontiguousarray(t, np.float32),
                             float(w), np.ascontiguousarray(r, np.int32), nb, tuples, phi, bucket)
    return tuples, phi, bucket


def lsh_hash_cosine(X, R):
    X = rows64(X)
    N, d = X.shape; L, k, _ = R.shape
    g = np.empty((N, L), np.int32)
    lib().or_lsh_hash_cosine(N, d, L, k, X, np.ascontiguousarray(R, np.float64), g)
    return g


def bucket_csr(bucket, nb):
    bucket = np.ascontiguousarray(bucket, np.int32)
    N, L = bucket.shape
    rp = np.empty((L, nb + 1), np.int64); idx = np.empty((L, N), np.int32)
    lib().or_bucket_csr(N, L, nb, bucket, rp, idx)
    return rp, idx


def lsh_query(N, nb, row_ptr, idx, q_bucket, tuples=None, q_tuple=None):
    L = row_ptr.shape[0]
    k = tuples.shape[2] if tuples is not None else 0
    qb = np.ascontiguousarray(q_bucket, np.int32)
    cap = int(sum(row_ptr[l, qb[l] + 1] - row_ptr[l, qb[l]] for l in range(L)))
    out = np.empty(max(cap, 1), np.int32)
    tu = None if tuples is None else np.ascontiguousarray(tuples, np.int32)
    qt = None if q_tuple is None else np.ascontiguousarray(q_tuple, np.int32)
    n = lib().or_lsh_query(N, L, k, nb, _ptr(tu), row_ptr, idx, _ptr(qt), qb, out, out.size)
    return out[:n].copy()


def cube_h(X, V, t, w):
    X = rows64(X)
    N, d = X.shape; k = t.shape[0]
    h = np.empty((N, k), np.int32)
    lib().or_cube_h(N, d, k, X, np.ascontiguousarray(V, np.float32), np.ascontiguousarray(t, np.float32), float(w), h)
    return h


class CoinMemo:
    """Dense per-f memo of the lazy Euclidean-F coins, plus the engine state."""

    def __init__(self, k, state, hmin=-(1 << 16), hspan=1 << 17):
        self.k, self.hmin, self.hspan = k, hmin, hspan
        self.memo = np.full((k, hspan), -1, np.int32)
        self.state = C.c_uint32(state)

    def apply(self, h):
        h = np.ascontiguousarray(h, np.int32)
        vertex = np.empty(h.shape[0], np.int32)
        n = lib().or_cube_coins(h.shape[0], self.k, h, self.hmin, self.hspan, self.memo, C.byref(self.state), vertex)
        if n < 0:
            raise ValueError("h outside memo span")
        return vertex, n

    def as_lists(self):
        f, off = np.nonzero(self.memo >= 0)
        return f.astype(np.int32), (off + self.hmin).astype(np.int32), self.memo[f, off].astype(np.int32)


def cube_cosine(X, R):
    X = rows64(X)
    N, d = X.shape; k = R.shape[0]
    v = np.empty(N, np.int32)
    lib().or_cube_cosine(N, d, k, X, np.ascontiguousarray(R, np.float64), v)
    return v


def cube_probe_seq(vertex, probes, k):
    cap = 1 << min(k, 24)
    out = np.empty(cap + 1, np.int32)
    n = lib().or_cube_probe_seq(int(vertex), int(probes), int(k), out, out.size)
    return out[:min(n, out.size)].copy()


def lloyd_assign(X, Cc, metric="euclidean", src_rows=None):
    X = rows64(X)
    Cc = np.ascontiguousarray(Cc, np.float64)
    N, d = X.shape; K = Cc.shape[0]
    a = np.empty(N, np.int32); dist = np.empty(N, np.float64)
    sr = None if src_rows is None else np.ascontiguousarray(src_rows, np.int32)
    lib().or_lloyd_assign(N, d, K, X, Cc, 0 if metric == "euclidean" else 1, _ptr(sr), a, dist)
    return a, dist


def range_assign(X, Cc, comb_ptr, comb_idx, metric="euclidean", key=None, src_rows=None):
    """range_assignment + lloyds_for_remaining + override (assignment.hpp:108-217).
    Returns (assign, dist, passes)."""
    X = rows64(X)
    Cc = np.ascontiguousarray(Cc, np.float64)
    N, d = X.shape; K = Cc.shape[0]
    a = np.empty(N, np.int32); dist = np.empty(N, np.float64)
    kk = None if key is None else np.ascontiguousarray(key, np.int32)
    sr = None if src_rows is None else np.ascontiguousarray(src_rows, np.int32)
    passes = lib().or_range_assign(N, d, K, X, Cc, 0 if metric == "euclidean" else 1,
                                   np.ascontiguousarray(comb_ptr, np.int64), np.ascontiguousarray(comb_idx, np.int32),
                                   _ptr(kk), _ptr(sr), a, dist)
    return a, dist, passes


def silhouette(X, assign, Cc, metric="euclidean"):
    """silhouette_cluster (silhouette.hpp:31-144): (sils [K+1], s [N])."""
    X = rows64(X)
    Cc = np.ascontiguousarray(Cc, np.float64)
    N, d = X.shape; K = Cc.shape[0]
    out = np.empty(K + 1, np.float64); s = np.empty(max(N, 1), np.float64)
    lib().or_silhouette(N, d, K, X, np.ascontiguousarray(assign, np.int32), Cc, 0 if metric == "euclidean" else 1,
                        out, _ptr(s))
    return out, s[:N]


def kmeans_update(X, assign, C_old, metric="euclidean", min_dist=0.0):
    X = rows64(X)
    N, d = X.shape; K = C_old.shape[0]
    Cn = np.empty((K, d), np.float64); cnt = np.empty(K, np.int64)
    cont = lib().or_kmeans_update(N, d, K, X, np.ascontiguousarray(assign, np.int32),
                                  np.ascontiguousarray(C_old, np.float64), 0 if metric == "euclidean" else 1,
                                  float(min_dist), Cn, cnt)
    return Cn, cnt, bool(cont)


def kmeans_pp(X, K, metric="euclidean", seed=1):
    """k_means_pp (initialization.hpp:71-156): the chosen rows."""
    X = rows64(X)
    N, d = X.shape
    rows = np.empty(K, np.int32)
    lib().or_kmeans_pp(N, d, K, X, 0 if metric == "euclidean" else 1, int(seed), rows)
    return rows


def rand_selection(N, K, seed=1):
    """rand_selection (initialization.hpp:39-69): the chosen rows."""
    rows = np.empty(K, np.int32)
    lib().or_rand_selection(int(seed), int(N), int(K), rows)
    return rows


def p_closest(X, U, cand_ptr, cand_idx, P):
    """get_P_closest (crypto_rec.hpp:213-231) per user: (idx [Q][P] -1-padded, sim [Q][P], cnt [Q])."""
    X = np.ascontiguousarray(X, np.float64); U = np.ascontiguousarray(U, np.float64)
    Q, d = U.shape
    idx = np.full((Q, P), -1, np.int32); sim = np.zeros((Q, P), np.float64); cnt = np.zeros(Q, np.int32)
    ci = np.ascontiguousarray(cand_idx, np.int32)
    lib().or_p_closest(d, X, Q, U, np.ascontiguousarray(cand_ptr, np.int64), ci if len(ci) else np.zeros(1, np.int32),
                       P, idx, sim, cnt)
    return idx, sim, cnt


def top_n_recom(X, x_mean, U, u_mean, unk_ptr, unk_idx, nb_idx, nb_sim, nb_cnt, N):
    """get_top_N_recom (crypto_rec.hpp:305-325) over get_P_closest lists: [Q][N], 0-padded."""
    X = np.ascontiguousarray(X, np.float64); U = np.ascontiguousarray(U, np.float64)
    Q, d = U.shape
    P = nb_idx.shape[1]
    out = np.zeros((Q, N), np.int32)
    ui = np.ascontiguousarray(unk_idx, np.int32)
    lib().or_top_n_recom(d, X, np.ascontiguousarray(x_mean, np.float64), Q, U, np.ascontiguousarray(u_mean, np.float64),
                         np.ascontiguousarray(unk_ptr, np.int64), ui if len(ui) else np.zeros(1, np.int32),
                         np.ascontiguousarray(nb_idx, np.int32), np.ascontiguousarray(nb_sim, np.float64),
                         np.ascontiguousarray(nb_cnt, np.int32), P, N, out)
    return out


def cluster_top_n(X, x_mean, crow, crows, U, u_mean, ucl, unk_ptr, unk_idx, N):
    """get_top_N_recom(neighbors, user, N) (crypto_rec.hpp:327-345) with each user's
    neighbours = the members of cluster ucl[q] (crows[crow[c]:crow[c+1]], member
    order), as main.cpp:260-269 / :353-373 call it: [Q][N], 0-padded; -1 rows for
    users of an empty cluster (main.cpp skips them)."""
    X = np.ascontiguousarray(X, np.float64); U = np.ascontiguousarray(U, np.float64)
    Q, d = U.shape
    out = np.zeros((Q, N), np.int32)
    ui = np.ascontiguousarray(unk_idx, np.int32)
    cr = np.ascontiguousarray(crows, np.int32)
    lib().or_cluster_top_n(d, X, np.ascontiguousarray(x_mean, np.float64), np.ascontiguousarray(crow, np.int64),
                           cr if len(cr) else np.zeros(1, np.int32), Q, U, np.ascontiguousarray(u_mean, np.float64),
                           np.ascontiguousarray(ucl, np.int32), np.ascontiguousarray(unk_ptr, np.int64),
                           ui if len(ui) else np.zeros(1, np.int32), N, out)
    return out


def clusters_csr(assign, K):
    """separate_clusters_from_input (utils.hpp:150-158): (crow [K+1], rows) in row order."""
    assign = np.asarray(assign, np.int64)
    order = np.argsort(assign, kind="stable").astype(np.int32)
    crow = np.zeros(K + 1, np.int64)
    np.add.at(crow, assign + 1, 1)
    return np.cumsum(crow), order
