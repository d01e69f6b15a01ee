"""Python binding of liblshkm (the MI355X LSH / hypercube / k-means hot path).

Thin ctypes layer over the C ABI in include/lshkm.h, used by the tests and
bench.py. Device buffers are torch tensors on a ROCm device (PyTorch is the
allocator and stream provider here, nothing more). The product is the HIP code
in csrc/: if liblshkm.so is missing this module raises — there is no CPU
fallback.

Reference-named entry points mirror lib/lsh_cube.hpp and
lib/clustering_phases/{assignment,update}.hpp (see the docstrings).
"""
import ctypes as C
import os
import re

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LSHKM_LIB") or os.path.join(_HERE, "liblshkm.so")   # override: profiling builds
HEADER = os.path.join(os.path.dirname(_HERE), "include", "lshkm.h")

EUCLIDEAN, COSINE = 0, 1
STAT_HASH_EXACT, STAT_ASSIGN_AMBIG, STAT_COS_FIX, STAT_REFINED, STAT_HASH_FIX, STAT_REC_SOFT = 0, 1, 4, 5, 6, 7
STAT_POW_FIX = 8
STAT_KM_SEQ = 9
_METRIC = {"euclidean": EUCLIDEAN, "cosine": COSINE, EUCLIDEAN: EUCLIDEAN, COSINE: COSINE}
DIST_CERTIFIED, DIST_EXACT = 0, 1
_DIST = {"certified": DIST_CERTIFIED, "default": DIST_CERTIFIED, "exact": DIST_EXACT,
         DIST_CERTIFIED: DIST_CERTIFIED, DIST_EXACT: DIST_EXACT}

_lib = None


class LshkmError(RuntimeError):
    pass


def pow_selfcheck():
    """Host only: the device's restatement of glibc's pow(x, 2) against this
    process's pow on discriminating inputs (lshkm_pow_selfcheck); returns
    (mismatches, tested)."""
    m, t = C.c_int64(), C.c_int64()
    _ck(lib().lshkm_pow_selfcheck(C.byref(m), C.byref(t)))
    return m.value, t.value


def declared_symbols():
    """Function names declared in include/lshkm.h."""
    with open(HEADER) as f:
        txt = f.read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(lshkm_\w+)\(", txt, re.M)))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LshkmError(f"{LIB_PATH} not built: run __graft_entry__.build() (no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        vp, i64, i32, u64, f32, f64 = C.c_void_p, C.c_int64, C.c_int, C.c_uint64, C.c_float, C.c_double
        sigs = {
            "lshkm_last_error": (C.c_char_p, []),
            "lshkm_version": (C.c_char_p, []),
            "lshkm_pow2": (i32, [vp, vp, i64, vp]),
            "lshkm_pow_selfcheck": (i32, [C.POINTER(i64), C.POINTER(i64)]),
            "lshkm_ctx_create": (i32, [i32, C.POINTER(vp)]),
            "lshkm_ctx_set_stream": (i32, [vp, vp]),
            "lshkm_ctx_set_dist_mode": (i32, [vp, i32]),
            "lshkm_ctx_get_dist_mode": (i32, [vp, C.POINTER(i32)]),
            "lshkm_ctx_sync": (i32, [vp]),
            "lshkm_ctx_destroy": (i32, [vp]),
            "lshkm_dev_alloc": (i32, [vp, i64, C.POINTER(vp)]),
            "lshkm_dev_free": (i32, [vp, vp]),
            "lshkm_memcpy_h2d": (i32, [vp, vp, vp, i64]),
            "lshkm_memcpy_d2h": (i32, [vp, vp, vp, i64]),
            "lshkm_get_stat": (i32, [vp, i32, C.POINTER(i64)]),
            "lshkm_reset_stats": (i32, [vp]),
            "lshkm_ctx_enable_timing": (i32, [vp, i32]),
            "lshkm_last_kernel_ms": (i32, [vp, C.POINTER(C.c_float)]),
            "lshkm_params_lsh_euclidean": (i32, [u64, i32, i32, i32, f32, vp, vp, vp, C.POINTER(C.c_uint32)]),
            "lshkm_params_lsh_cosine": (i32, [u64, i32, i32, i32, vp, C.POINTER(C.c_uint32)]),
            "lshkm_params_cube_euclidean": (i32, [u64, i32, i32, f32, vp, vp, C.POINTER(C.c_uint32)]),
            "lshkm_params_cube_cosine": (i32, [u64, i32, i32, vp, C.POINTER(C.c_uint32)]),
            "lshkm_lsh_create": (i32, [vp, i32, i32, i32, i32, i64, f32, vp, vp, vp, vp, C.POINTER(vp)]),
            "lshkm_lsh_destroy": (i32, [vp]),
            "lshkm_lsh_hash": (i32, [vp, vp, i64, vp, vp, vp]),
            "lshkm_lsh_build": (i32, [vp, vp, i64]),
            "lshkm_lsh_get_buckets": (i32, [vp, i32, vp, vp]),
            "lshkm_lsh_device_views": (i32, [vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.POINTER(vp)]),
            "lshkm_lsh_query": (i32, [vp, vp, i64, vp, i32, vp, vp, i64, C.POINTER(i64)]),
            "lshkm_cube_create": (i32, [vp, i32, i32, i32, f32, vp, vp, vp, C.c_uint32, C.POINTER(vp)]),
            "lshkm_cube_destroy": (i32, [vp]),
            "lshkm_cube_build": (i32, [vp, vp, i64]),
            "lshkm_cube_vertices": (i32, [vp, vp, i64, vp]),
            "lshkm_cube_get_buckets": (i32, [vp, vp, vp]),
            "lshkm_cube_query": (i32, [vp, vp, i64, i32, vp, vp, i64, C.POINTER(i64)]),
            "lshkm_cube_get_memo": (i32, [vp, vp, vp, vp, i64, C.POINTER(i64), C.POINTER(C.c_uint32)]),
            "lshkm_cube_unseen": (i32, [vp, vp, i64, vp, vp, vp, i64, C.POINTER(i64)]),
            "lshkm_cube_import_coins": (i32, [vp, vp, vp, vp, i64, C.c_uint32]),
            "lshkm_coins_draw": (i32, [C.POINTER(C.c_uint32), vp, i64, vp]),
            "lshkm_lloyd_assign": (i32, [vp, vp, i64, i32, vp, i32, i32, vp, vp, vp]),
            "lshkm_range_assign": (i32, [vp, vp, i64, i32, vp, i32, i32, vp, vp, vp, vp, vp, vp, C.POINTER(i32)]),
            "lshkm_silhouette": (i32, [vp, vp, i64, i32, vp, vp, i32, i32, vp, vp]),
            "lshkm_vectors_read": (i32, [C.c_char_p, C.c_char, i32, i32, C.POINTER(vp)]),
            "lshkm_vectors_info": (i32, [vp, C.POINTER(i64), C.POINTER(i32), C.POINTER(i64), C.POINTER(i32),
                                         C.POINTER(i32), C.POINTER(i32)]),
            "lshkm_vectors_values": (i32, [vp, vp, vp]),
            "lshkm_vectors_ids": (i32, [vp, vp, vp]),
            "lshkm_vectors_meta": (i32, [vp, i32, C.c_char_p, i64, C.POINTER(i64)]),
            "lshkm_vectors_free": (i32, [vp]),
            "lshkm_config_value": (i32, [C.c_char_p, C.c_char_p, C.c_char_p, i64, C.POINTER(i32)]),
            "lshkm_config_load": (i32, [C.c_char_p, vp]),
            "lshkm_hash_assign": (i32, [vp, vp, i64, vp, i32, vp, vp, vp, vp, vp, vp]),
            "lshkm_hash_assign_metric": (i32, [vp, vp, i64, vp, i32, i32, vp, vp, vp, vp, vp, vp]),
            "lshkm_kmeans_update": (i32, [vp, vp, i64, i32, vp, vp, i32, i32, f64, vp, vp, C.POINTER(i32)]),
            "lshkm_kmeans_partial": (i32, [vp, vp, i64, i32, vp, i32, vp, vp]),
            "lshkm_kmeans_partial_carry": (i32, [vp, vp, i64, i32, vp, i32, vp, vp, vp, vp]),
            "lshkm_kmeans_partial_csr": (i32, [vp, vp, i64, i32, vp, vp, i32, vp, vp]),
            "lshkm_kmeans_finalize": (i32, [vp, vp, vp, i32, i32, vp, i32, f64, vp, C.POINTER(i32)]),
            "lshkm_kmeans_shard_begin": (i32, [vp, vp, i64, i32, vp, vp, i32, vp, vp, vp, vp]),
            "lshkm_kmeans_shard_certify": (i32, [vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp,
                                                 C.POINTER(i64)]),
            "lshkm_kmeans_shard_ws_bytes": (i32, [i64, i32, i32, C.POINTER(i64)]),
            "lshkm_kmeans_shard_prepare": (i32, [vp, vp, i64, i32, vp, vp, i32, vp, vp, vp, vp, i64]),
            "lshkm_kmeans_shard_chain": (i32, [vp, vp, i64, i32, vp, vp, i32, vp, vp, vp, vp, i64, vp]),
            "lshkm_kmeans_pp": (i32, [vp, vp, i64, i32, i32, i32, u64, vp]),
            "lshkm_rand_selection": (i32, [u64, i64, i32, vp]),
            "lshkm_p_closest": (i32, [vp, vp, i64, i32, vp, i64, vp, vp, i32, vp, vp, vp]),
            "lshkm_top_n_recom": (i32, [vp, vp, vp, i64, i32, vp, i64, vp, vp, vp, vp, vp, i32, i32, vp]),
            "lshkm_cluster_top_n": (i32, [vp, vp, vp, i64, i32, vp, vp, i32, vp, vp, i64, vp, vp, vp, i32, vp]),
            "lshkm_cluster_sims": (i32, [vp, vp, i64, i32, vp, vp, i32, vp, i64, vp, vp, vp, vp, i64,
                                         C.POINTER(i64)]),
            "lshkm_cluster_chain": (i32, [vp, vp, vp, i64, i32, vp, vp, i32, i64, vp, vp, vp, vp, vp, vp, vp, vp,
                                          vp, vp, vp, vp, i32, vp]),
            "lshkm_cluster_terms": (i32, [vp, vp, vp, i64, i32, vp, vp, i32, vp, i64, vp, vp, vp, vp, vp, vp, vp,
                                          i64, i64, C.POINTER(i64), C.POINTER(i64)]),
            "lshkm_cluster_chain_terms": (i32, [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32,
                                                vp]),
            "lshkm_synth": (i32, [vp, u64, i64, i64, i32, vp]),
            "lshkm_synth_normal": (i32, [vp, u64, i64, i64, i32, vp]),
            "lshkm_clusters": (i32, [vp, vp, i64, i32, vp, vp]),
        }
        for name, (res, args) in sigs.items():
            for nm in (name, name + "_f64"):     # fp64-row twins share the signature
                if not hasattr(L, nm):
                    continue   # reported by tests/test_lib_cpu.py::test_exports
                fn = getattr(L, nm)
                fn.restype = res
                fn.argtypes = args
        _lib = L
    return _lib


def _ck(rc):
    if rc != 0:
        raise LshkmError(f"lshkm error {rc}: {lib().lshkm_last_error().decode()}")


def _np_ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _t_ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


# Entry points that read dataset rows exist for fp32 rows (name) and fp64 rows
# (name_f64, SURVEY §8a: general doubles such as the recommender's user
# vectors); the rows' dtype picks one.
def _fn(name, X):
    dt = str(X.dtype)
    if dt.endswith("float32"):
        return getattr(lib(), name)
    if dt.endswith("float64"):
        return getattr(lib(), name + "_f64")
    raise LshkmError(f"{name}: rows must be float32 or float64, got {dt}")


# ------------------------------------------------------------------ parameters
def params_lsh_euclidean(seed, L, k, d, w):
    V = np.empty((L, k, d), np.float32); t = np.empty((L, k), np.float32); r = np.empty((L, k), np.int32)
    st = C.c_uint32()
    _ck(lib().lshkm_params_lsh_euclidean(seed, L, k, d, float(np.float32(w)), _np_ptr(V), _np_ptr(t), _np_ptr(r), C.byref(st)))
    return V, t, r, st.value


def params_lsh_cosine(seed, L, k, d):
    R = np.empty((L, k, d), np.float64); st = C.c_uint32()
    _ck(lib().lshkm_params_lsh_cosine(seed, L, k, d, _np_ptr(R), C.byref(st)))
    return R, st.value


def params_cube_euclidean(seed, k, d, w):
    V = np.empty((k, d), np.float32); t = np.empty((k,), np.float32); st = C.c_uint32()
    _ck(lib().lshkm_params_cube_euclidean(seed, k, d, float(np.float32(w)), _np_ptr(V), _np_ptr(t), C.byref(st)))
    return V, t, st.value


def params_cube_cosine(seed, k, d):
    R = np.empty((k, d), np.float64); st = C.c_uint32()
    _ck(lib().lshkm_params_cube_cosine(seed, k, d, _np_ptr(R), C.byref(st)))
    return R, st.value


# --------------------------------------------------------------------- context
class Context:
    def __init__(self, device=0, use_torch_stream=True):
        import torch
        self.torch = torch
        self.device = device
        self.dev = torch.device("cuda", device)
        h = C.c_void_p()
        _ck(lib().lshkm_ctx_create(device, C.byref(h)))
        self.h = h
        if use_torch_stream:
            _ck(lib().lshkm_ctx_set_stream(self.h, C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)))

    def set_dist_mode(self, mode):
        """The context's distance contract (lshkm_ctx_set_dist_mode): "certified"
        (the default: euclidean winner distances within 2^-20 relative) or
        "exact" (the reference's fp64 chain for every distance)."""
        _ck(lib().lshkm_ctx_set_dist_mode(self.h, _DIST[mode]))

    def pow2(self, x):
        """pow(x, 2) as the reference's glibc computes it (lshkm_pow2), for a
        float64 device tensor."""
        x = x.contiguous()
        assert x.dtype == self.torch.float64 and x.device.type == "cuda"
        out = self.torch.empty_like(x)
        _ck(lib().lshkm_pow2(self.h, C.c_void_p(x.data_ptr()), x.numel(), C.c_void_p(out.data_ptr())))
        return out

    def dist_mode(self):
        m = C.c_int()
        _ck(lib().lshkm_ctx_get_dist_mode(self.h, C.byref(m)))
        return "exact" if m.value == DIST_EXACT else "certified"

    def sync(self):
        _ck(lib().lshkm_ctx_sync(self.h))

    def stat(self, which):
        v = C.c_int64()
        _ck(lib().lshkm_get_stat(self.h, which, C.byref(v)))
        return v.value

    def reset_stats(self):
        _ck(lib().lshkm_reset_stats(self.h))

    def close(self):
        if self.h:
            lib().lshkm_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def empty(self, shape, dtype):
        return self.torch.empty(shape, dtype=dtype, device=self.dev)

    def synth(self, seed, rows, d, row0=0, kind="grid"):
        """include/lshkm_synth.h rows on the device: kind "grid" (the default,
        2^-15 grid) or "normal" (Irwin-Hall(12), full fp32 mantissas)."""
        X = self.empty((rows, d), self.torch.float32)
        fn = {"grid": lib().lshkm_synth, "normal": lib().lshkm_synth_normal}[kind]
        _ck(fn(self.h, seed, row0, rows, d, _t_ptr(X)))
        return X


# ------------------------------------------------------------------------ LSH
class LSH:
    """A set of L hashtables (create_LSH_hashtables, lsh_cube.hpp:44-74)."""

    def __init__(self, ctx, metric, d, k, L, nb=0, w=0.0, V=None, t=None, r=None, R=None):
        self.ctx, self.metric, self.d, self.k, self.L = ctx, _METRIC[metric], d, k, L
        self.nb = nb if self.metric == EUCLIDEAN else (1 << k)
        self.w = float(np.float32(w))
        keep = [np.ascontiguousarray(a, dt) if a is not None else None
                for a, dt in ((V, np.float32), (t, np.float32), (r, np.int32), (R, np.float64))]
        h = C.c_void_p()
        _ck(lib().lshkm_lsh_create(ctx.h, self.metric, d, k, L, self.nb, self.w, *[_np_ptr(a) for a in keep], C.byref(h)))
        self.h = h
        self.N = 0

    def close(self):
        if self.h:
            lib().lshkm_lsh_destroy(self.h)
            self.h = None
        self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def hash(self, X, tuples=True, phi=True, bucket=True):
        torch = self.ctx.torch
        N = X.shape[0]
        tu = self.ctx.empty((N, self.L, self.k), torch.int32) if (tuples and self.metric == EUCLIDEAN) else None
        ph = self.ctx.empty((N, self.L), torch.int32) if phi else None
        bu = self.ctx.empty((N, self.L), torch.int32) if bucket else None
        _ck(_fn("lshkm_lsh_hash", X)(self.h, _t_ptr(X), N, _t_ptr(tu), _t_ptr(ph), _t_ptr(bu)))
        return tu, ph, bu

    def build(self, X):
        _ck(_fn("lshkm_lsh_build", X)(self.h, _t_ptr(X), X.shape[0]))
        self.N = X.shape[0]

    def buckets(self, table):
        rp = np.empty(self.nb + 1, np.int64); idx = np.empty(max(self.N, 1), np.int32)
        _ck(lib().lshkm_lsh_get_buckets(self.h, table, _np_ptr(rp), _np_ptr(idx)))
        return rp, idx[:self.N]

    def query(self, Q, filtered=True, alias_rows=None, device=False):
        """Batched get_LSH_[filtered_]combined_buckets: returns (ptr[nq+1], idx) numpy."""
        torch = self.ctx.torch
        nq = Q.shape[0]
        ptr = self.ctx.empty((nq + 1,), torch.int64)
        total = C.c_int64()
        _ck(_fn("lshkm_lsh_query", Q)(self.h, _t_ptr(Q), nq, _t_ptr(alias_rows), int(filtered), _t_ptr(ptr), None, 0,
                                  C.byref(total)))
        out = self.ctx.empty((max(total.value, 1),), torch.int32)
        _ck(_fn("lshkm_lsh_query", Q)(self.h, _t_ptr(Q), nq, _t_ptr(alias_rows), int(filtered), _t_ptr(ptr), _t_ptr(out),
                                  total.value, C.byref(total)))
        self.ctx.sync()
        if device:                                   # device tensors, no host copy
            return ptr, out[:total.value]
        return ptr.cpu().numpy(), out[:total.value].cpu().numpy()


class Cube:
    """The randomized hypercube (create_hypercube, lsh_cube.hpp:108-136)."""

    def __init__(self, ctx, metric, d, k, w=0.0, V=None, t=None, R=None, rng_state=1):
        self.ctx, self.metric, self.d, self.k = ctx, _METRIC[metric], d, k
        keep = [np.ascontiguousarray(a, dt) if a is not None else None
                for a, dt in ((V, np.float32), (t, np.float32), (R, np.float64))]
        h = C.c_void_p()
        _ck(lib().lshkm_cube_create(ctx.h, self.metric, d, k, float(np.float32(w)), *[_np_ptr(a) for a in keep],
                                    rng_state, C.byref(h)))
        self.h = h
        self.N = 0

    def close(self):
        if self.h:
            lib().lshkm_cube_destroy(self.h)
            self.h = None
        self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def build(self, X):
        _ck(_fn("lshkm_cube_build", X)(self.h, _t_ptr(X), X.shape[0]))
        self.N = X.shape[0]

    def vertices(self, Q):
        v = self.ctx.empty((Q.shape[0],), self.ctx.torch.int32)
        _ck(_fn("lshkm_cube_vertices", Q)(self.h, _t_ptr(Q), Q.shape[0], _t_ptr(v)))
        return v

    def buckets(self):
        rp = np.empty((1 << self.k) + 1, np.int64); idx = np.empty(max(self.N, 1), np.int32)
        _ck(lib().lshkm_cube_get_buckets(self.h, _np_ptr(rp), _np_ptr(idx)))
        return rp, idx[:self.N]

    def memo(self):
        cnt = C.c_int64(); st = C.c_uint32()
        _ck(lib().lshkm_cube_get_memo(self.h, None, None, None, 0, C.byref(cnt), C.byref(st)))
        n = cnt.value
        f = np.empty(max(n, 1), np.int32); hh = np.empty(max(n, 1), np.int32); b = np.empty(max(n, 1), np.int32)
        _ck(lib().lshkm_cube_get_memo(self.h, _np_ptr(f), _np_ptr(hh), _np_ptr(b), n, C.byref(cnt), C.byref(st)))
        return f[:n], hh[:n], b[:n], st.value

    def unseen(self, X):
        """(f, h, first local row) of the (f, h) pairs in X without a coin yet (lshkm_cube_unseen)."""
        cnt = C.c_int64()
        _ck(_fn("lshkm_cube_unseen", X)(self.h, _t_ptr(X), X.shape[0], None, None, None, 0, C.byref(cnt)))
        n = cnt.value
        f = np.empty(max(n, 1), np.int32); hh = np.empty(max(n, 1), np.int32); r = np.empty(max(n, 1), np.int64)
        _ck(_fn("lshkm_cube_unseen", X)(self.h, _t_ptr(X), X.shape[0], _np_ptr(f), _np_ptr(hh), _np_ptr(r), n,
                                    C.byref(cnt)))
        return f[:n], hh[:n], r[:n]

    def import_coins(self, f, h, bits, rng_state):
        f, h, bits = (np.ascontiguousarray(a, np.int32) for a in (f, h, bits))
        _ck(lib().lshkm_cube_import_coins(self.h, _np_ptr(f), _np_ptr(h), _np_ptr(bits), len(f), rng_state))

    def query(self, Q, probes, device=False):
        torch = self.ctx.torch
        nq = Q.shape[0]
        ptr = self.ctx.empty((nq + 1,), torch.int64)
        total = C.c_int64()
        _ck(_fn("lshkm_cube_query", Q)(self.h, _t_ptr(Q), nq, probes, _t_ptr(ptr), None, 0, C.byref(total)))
        out = self.ctx.empty((max(total.value, 1),), torch.int32)
        _ck(_fn("lshkm_cube_query", Q)(self.h, _t_ptr(Q), nq, probes, _t_ptr(ptr), _t_ptr(out), total.value,
                                   C.byref(total)))
        self.ctx.sync()
        if device:                                   # device tensors, no host copy
            return ptr, out[:total.value]
        return ptr.cpu().numpy(), out[:total.value].cpu().numpy()


def coins_draw(rng_state, h):
    """Host EuclideanF coins in order (lshkm_coins_draw): returns (bits, new state)."""
    h = np.ascontiguousarray(h, np.int32)
    bits = np.empty(max(len(h), 1), np.int32)
    st = C.c_uint32(rng_state)
    _ck(lib().lshkm_coins_draw(C.byref(st), _np_ptr(h), len(h), _np_ptr(bits)))
    return bits[:len(h)], st.value


# -------------------------------------------------------------------- k-means
def lloyd_assign(ctx, X, Cc, metric="euclidean", src_rows=None, assign=None, dist=None):
    """lloyds_assignment (assignment.hpp:54-80). Returns (assign int32, dist fp64) tensors."""
    torch = ctx.torch
    N, d = X.shape
    K = Cc.shape[0]
    assign = ctx.empty((N,), torch.int32) if assign is None else assign
    dist = ctx.empty((N,), torch.float64) if dist is None else dist
    sr = None if src_rows is None else np.ascontiguousarray(src_rows, np.int32)
    _ck(_fn("lshkm_lloyd_assign", X)(ctx.h, _t_ptr(X), N, d, _t_ptr(Cc), K, _METRIC[metric], _np_ptr(sr),
                                 _t_ptr(assign), _t_ptr(dist)))
    return assign, dist


def range_assign(ctx, X, Cc, comb_ptr, comb_idx, metric="euclidean", key=None, src_rows=None):
    """lsh_range_assignment / cube_range_assignment (assignment.hpp:108-145) over
    the centroids' combined buckets (device or host CSR). Returns (assign, dist, passes)."""
    torch = ctx.torch
    N, d = X.shape
    K = Cc.shape[0]
    cp = torch.as_tensor(np.ascontiguousarray(comb_ptr, np.int64)).to(ctx.dev) if isinstance(comb_ptr, np.ndarray) else comb_ptr
    ci = torch.as_tensor(np.ascontiguousarray(comb_idx, np.int32)).to(ctx.dev) if isinstance(comb_idx, np.ndarray) else comb_idx
    if ci.numel() == 0:
        ci = ctx.empty((1,), torch.int32)
    assign = ctx.empty((N,), torch.int32)
    dist = ctx.empty((N,), torch.float64)
    kk = None if key is None else np.ascontiguousarray(key, np.int32)
    sr = None if src_rows is None else np.ascontiguousarray(src_rows, np.int32)
    passes = C.c_int32(0)
    _ck(_fn("lshkm_range_assign", X)(ctx.h, _t_ptr(X), N, d, _t_ptr(Cc), K, _METRIC[metric], _t_ptr(cp), _t_ptr(ci),
                                 _np_ptr(kk), _np_ptr(sr), _t_ptr(assign), _t_ptr(dist), C.byref(passes)))
    return assign, dist, passes.value


def silhouette(ctx, X, assign, Cc, metric="euclidean"):
    """silhouette_cluster (silhouette.hpp:31-80). Returns (sils [K+1] numpy, s [N] tensor)."""
    N, d = X.shape
    K = Cc.shape[0]
    out = np.empty(K + 1, np.float64)
    s = ctx.empty((max(N, 1),), ctx.torch.float64)
    _ck(_fn("lshkm_silhouette", X)(ctx.h, _t_ptr(X), N, d, _t_ptr(assign), _t_ptr(Cc), K, _METRIC[metric], _np_ptr(out),
                               _t_ptr(s)))
    return out, s[:N]


# ------------------------------------------------------------- input formats
class Config(C.Structure):
    """lshkm_config: get_config's values (main.cpp:512-554)."""
    _fields_ = [("proj_2_input", C.c_char * 1024), ("proj_2_csv_delimiter", C.c_char), ("proj_2_cluster_num", C.c_int32),
                ("cluster_num", C.c_int32), ("has_cluster_num", C.c_int32), ("k", C.c_int32), ("L", C.c_int32),
                ("lsh_bucket_div", C.c_int32), ("euclidean_h_w", C.c_double), ("csv_delimiter", C.c_char),
                ("max_algo_iterations", C.c_int32), ("min_dist_kmeans", C.c_double),
                ("lexicon_file", C.c_char * 1024), ("query_file", C.c_char * 1024)]


def load_config(path):
    c = Config()
    _ck(lib().lshkm_config_load(path.encode(), C.byref(c)))
    return c


def config_value(path, key):
    buf = C.create_string_buffer(4096)
    found = C.c_int32(0)
    _ck(lib().lshkm_config_value(path.encode(), key.encode(), buf, len(buf), C.byref(found)))
    return buf.value.decode() if found.value else None


def read_vectors(path, delimiter=",", strt_line=1, threads=0):
    """VectorReader<double>::read (vector_reader.hpp:54-85): (ids list, X fp64 [n][d],
    fp32_exact flag, metadata lines)."""
    h = C.c_void_p()
    _ck(lib().lshkm_vectors_read(path.encode(), delimiter.encode()[:1], strt_line, threads, C.byref(h)))
    try:
        n, d, ib, rg, ex, nm = C.c_int64(), C.c_int32(), C.c_int64(), C.c_int32(), C.c_int32(), C.c_int32()
        _ck(lib().lshkm_vectors_info(h, C.byref(n), C.byref(d), C.byref(ib), C.byref(rg), C.byref(ex), C.byref(nm)))
        if rg.value:
            raise LshkmError("ragged rows: no N x d layout")
        X = np.empty((n.value, d.value), np.float64)
        _ck(lib().lshkm_vectors_values(h, _np_ptr(X), None))
        raw = C.create_string_buffer(max(ib.value, 1))
        off = np.empty(n.value + 1, np.int64)
        _ck(lib().lshkm_vectors_ids(h, raw, _np_ptr(off)))
        b = raw.raw
        ids = [b[off[i]:off[i + 1]].decode() for i in range(n.value)]
        meta = []
        for i in range(nm.value):
            ln = C.c_int64()
            _ck(lib().lshkm_vectors_meta(h, i, None, 0, C.byref(ln)))
            buf = C.create_string_buffer(ln.value + 1)
            _ck(lib().lshkm_vectors_meta(h, i, buf, len(buf), None))
            meta.append(buf.value.decode())
        return ids, X, bool(ex.value), meta
    finally:
        lib().lshkm_vectors_free(h)


def hash_assign(lsh, X, Cc, src_rows=None, tuples=True, phi=False, bucket=True, metric=None):
    """LSH hashing + Lloyd assignment in one pass. Returns (tuples, phi, bucket, assign, dist).
    metric None: euclidean Lloyd (lshkm_hash_assign); else the assignment metric
    (lshkm_hash_assign_metric: a cosine index with cosine Lloyd is one pass)."""
    ctx, torch = lsh.ctx, lsh.ctx.torch
    N = X.shape[0]
    tu = ctx.empty((N, lsh.L, lsh.k), torch.int32) if (tuples and lsh.metric == EUCLIDEAN) else None
    ph = ctx.empty((N, lsh.L), torch.int32) if phi else None
    bu = ctx.empty((N, lsh.L), torch.int32) if bucket else None
    a = ctx.empty((N,), torch.int32)
    dist = ctx.empty((N,), torch.float64)
    sr = None if src_rows is None else np.ascontiguousarray(src_rows, np.int32)
    if metric is None:
        _ck(_fn("lshkm_hash_assign", X)(lsh.h, _t_ptr(X), N, _t_ptr(Cc), Cc.shape[0], _np_ptr(sr), _t_ptr(tu),
                                        _t_ptr(ph), _t_ptr(bu), _t_ptr(a), _t_ptr(dist)))
    else:
        _ck(_fn("lshkm_hash_assign_metric", X)(lsh.h, _t_ptr(X), N, _t_ptr(Cc), Cc.shape[0], _METRIC[metric],
                                               _np_ptr(sr), _t_ptr(tu), _t_ptr(ph), _t_ptr(bu), _t_ptr(a),
                                               _t_ptr(dist)))
    return tu, ph, bu, a, dist


def kmeans_update(ctx, X, assign, C_old, metric="euclidean", min_dist=0.0):
    """k_means (update.hpp:37-86). Returns (C_new, counts, cont)."""
    torch = ctx.torch
    N, d = X.shape
    K = C_old.shape[0]
    Cn = ctx.empty((K, d), torch.float64)
    cnt = ctx.empty((K,), torch.int64)
    cont = C.c_int()
    _ck(_fn("lshkm_kmeans_update", X)(ctx.h, _t_ptr(X), N, d, _t_ptr(assign), _t_ptr(C_old), K, _METRIC[metric],
                                  float(min_dist), _t_ptr(Cn), _t_ptr(cnt), C.byref(cont)))
    return Cn, cnt, bool(cont.value)


def kmeans_partial(ctx, X, assign, K, sums=None, counts=None, csr=None):
    """Per-shard exact sums (lshkm_kmeans_partial); csr = (crow, rows) of this
    assignment from clusters(): lshkm_kmeans_partial_csr, no second sort."""
    torch = ctx.torch
    N, d = X.shape
    sums = ctx.empty((K, d), torch.float64) if sums is None else sums
    counts = ctx.empty((K,), torch.int64) if counts is None else counts
    if csr is not None:
        _ck(_fn("lshkm_kmeans_partial_csr", X)(ctx.h, _t_ptr(X), N, d, _t_ptr(csr[0]), _t_ptr(csr[1]), K, _t_ptr(sums),
                                               _t_ptr(counts)))
    else:
        _ck(_fn("lshkm_kmeans_partial", X)(ctx.h, _t_ptr(X), N, d, _t_ptr(assign), K, _t_ptr(sums), _t_ptr(counts)))
    return sums, counts


def kmeans_partial_carry(ctx, X, assign, K, carry_sums=None, carry_counts=None):
    """Exact-mode shard update: the chains continue from the previous shard's
    (sums, counts) -- None for the first shard (lshkm_kmeans_partial_carry)."""
    torch = ctx.torch
    N, d = X.shape
    sums = ctx.empty((K, d), torch.float64)
    counts = ctx.empty((K,), torch.int64)
    _ck(_fn("lshkm_kmeans_partial_carry", X)(ctx.h, _t_ptr(X), N, d, _t_ptr(assign), K,
                                         _t_ptr(carry_sums) if carry_sums is not None else None,
                                         _t_ptr(carry_counts) if carry_counts is not None else None,
                                         _t_ptr(sums), _t_ptr(counts)))
    return sums, counts


class ShardSums:
    """One rank's part of the sharded exact k-means sums (lshkm_kmeans_shard_*,
    include/lshkm.h): X this rank's rows, csr = (crow, rows) of its assignment
    (clusters()). sharding.kmeans_sums_sharded runs the exchange between the
    calls; every method works on device tensors."""

    def __init__(self, ctx, X, csr, K):
        self.ctx, self.X, self.csr, self.K = ctx, X, csr, K
        self.N, self.d = X.shape
        self.ws = None

    def empty(self, shape, dtype):
        return self.ctx.empty(shape, dtype)

    def begin(self):
        """-> (sums [K][d], asum [K][d], qt [2][K][d] int32, counts [K]): this rank's partials."""
        torch, K, d = self.ctx.torch, self.K, self.d
        sums, asum = self.empty((K, d), torch.float64), self.empty((K, d), torch.float64)
        qt, counts = self.empty((2, K, d), torch.int32), self.empty((K,), torch.int64)
        _ck(_fn("lshkm_kmeans_shard_begin", self.X)(self.ctx.h, _t_ptr(self.X), self.N, d, _t_ptr(self.csr[0]),
                                                    _t_ptr(self.csr[1]), K, _t_ptr(sums), _t_ptr(asum), _t_ptr(qt),
                                                    _t_ptr(counts)))
        return sums, asum, qt, counts

    def certify(self, gathered, asum, qt, counts, world, rank):
        """-> (sums_out, start, flag, mask, n_flagged) from the exchanged values."""
        torch, K, d = self.ctx.torch, self.K, self.d
        out, start = self.empty((K, d), torch.float64), self.empty((K, d), torch.float64)
        flag, mask = self.empty((K,), torch.int32), self.empty((K, d), torch.uint8)
        nf = C.c_int64()
        _ck(lib().lshkm_kmeans_shard_certify(self.ctx.h, K, d, world, rank, _t_ptr(gathered), _t_ptr(asum),
                                             _t_ptr(qt), _t_ptr(counts), _t_ptr(out), _t_ptr(start), _t_ptr(flag),
                                             _t_ptr(mask), C.byref(nf)))
        return out, start, flag, mask, int(nf.value)

    def _ws(self):
        nb = C.c_int64()
        _ck(lib().lshkm_kmeans_shard_ws_bytes(self.N, self.K, self.d, C.byref(nb)))
        if self.ws is None or self.ws.numel() < nb.value:
            self.ws = self.empty((int(nb.value),), self.ctx.torch.uint8)
        return self.ws

    def prepare(self, start, flag, mask):
        ws = self._ws()
        _ck(_fn("lshkm_kmeans_shard_prepare", self.X)(self.ctx.h, _t_ptr(self.X), self.N, self.d, _t_ptr(self.csr[0]),
                                                      _t_ptr(self.csr[1]), self.K, _t_ptr(start), _t_ptr(flag),
                                                      _t_ptr(mask), _t_ptr(ws), ws.numel()))

    def chain(self, flag, mask, carry, sums):
        ws = self._ws()
        _ck(_fn("lshkm_kmeans_shard_chain", self.X)(self.ctx.h, _t_ptr(self.X), self.N, self.d, _t_ptr(self.csr[0]),
                                                    _t_ptr(self.csr[1]), self.K, _t_ptr(flag), _t_ptr(mask),
                                                    _t_ptr(carry) if carry is not None else None, _t_ptr(ws),
                                                    ws.numel(), _t_ptr(sums)))


def kmeans_finalize(ctx, sums, counts, C_old, metric="euclidean", min_dist=0.0):
    torch = ctx.torch
    K, d = sums.shape
    Cn = ctx.empty((K, d), torch.float64)
    cont = C.c_int()
    _ck(lib().lshkm_kmeans_finalize(ctx.h, _t_ptr(sums), _t_ptr(counts), K, d, _t_ptr(C_old), _METRIC[metric],
                                    float(min_dist), _t_ptr(Cn), C.byref(cont)))
    return Cn, bool(cont.value)


def kmeans_pp_rows(ctx, X, K, metric="euclidean", seed=1):
    """k_means_pp (initialization.hpp:71-156): the K chosen dataset rows (int32 numpy)."""
    N, d = X.shape
    rows = np.empty(K, np.int32)
    _ck(_fn("lshkm_kmeans_pp", X)(ctx.h, _t_ptr(X), N, d, K, _METRIC[metric], int(seed), _np_ptr(rows)))
    return rows


def clusters(ctx, assign, K):
    """separate_clusters_from_input (utils.hpp:150-158): the member lists of the K
    clusters as a CSR (crow [K+1] int64, rows [N] int32 device tensors; members
    in row order)."""
    torch = ctx.torch
    N = assign.shape[0]
    crow = ctx.empty((K + 1,), torch.int64)
    rows = ctx.empty((max(N, 1),), torch.int32)
    _ck(lib().lshkm_clusters(ctx.h, _t_ptr(assign), N, K, _t_ptr(crow), _t_ptr(rows)))
    return crow, rows[:N]


def rand_selection_rows(N, K, seed=1):
    """rand_selection (initialization.hpp:39-69): K distinct rows (host only)."""
    rows = np.empty(K, np.int32)
    _ck(lib().lshkm_rand_selection(int(seed), int(N), int(K), _np_ptr(rows)))
    return rows


# ------------------------------------------------------------ recommendation
def p_closest(ctx, X, U, cand_ptr, cand_idx, P):
    """get_P_closest (crypto_rec.hpp:213-231) for all users of U at once.
    X [N][d], U [nq][d] fp64 device tensors; cand_ptr [nq+1] int64 / cand_idx
    int32 device tensors. Returns (idx [nq][P] -1-padded, sim [nq][P], cnt [nq])."""
    torch = ctx.torch
    N, d = X.shape
    nq = U.shape[0]
    idx = ctx.empty((nq, P), torch.int32)
    sim = ctx.empty((nq, P), torch.float64)
    cnt = ctx.empty((nq,), torch.int32)
    _ck(lib().lshkm_p_closest(ctx.h, _t_ptr(X), N, d, _t_ptr(U), nq, _t_ptr(cand_ptr),
                              _t_ptr(cand_idx) if cand_idx.numel() else None, P, _t_ptr(idx), _t_ptr(sim),
                              _t_ptr(cnt)))
    return idx, sim, cnt


def top_n_recom(ctx, X, x_mean, u_mean, unk_ptr, unk_idx, nb_idx, nb_sim, nb_cnt, n_top):
    """get_top_N_recom (crypto_rec.hpp:305-325) over p_closest's lists: [nq][n_top] int32."""
    torch = ctx.torch
    N, d = X.shape
    nq, P = nb_idx.shape
    out = ctx.empty((nq, n_top), torch.int32)
    _ck(lib().lshkm_top_n_recom(ctx.h, _t_ptr(X), _t_ptr(x_mean), N, d, _t_ptr(u_mean), nq, _t_ptr(unk_ptr),
                                _t_ptr(unk_idx) if unk_idx.numel() else None, _t_ptr(nb_idx), _t_ptr(nb_sim),
                                _t_ptr(nb_cnt), P, n_top, _t_ptr(out)))
    return out


def cluster_top_n(ctx, X, x_mean, crow, crows, U, u_mean, ucl, unk_ptr, unk_idx, n_top):
    """get_top_N_recom(neighbors, user, N) (crypto_rec.hpp:327-345) for every user
    of U, its neighbours = the members of cluster ucl[q] (crow [K+1] int64 /
    crows int32, lshkm_clusters' CSR), as main.cpp:260-269 / :353-373 call it.
    X [N][d] / U [nq][d] rows of one dtype (fp32 or fp64), means fp64, all device
    tensors. Returns [nq][n_top] int32 (0-padded; -1 rows: empty cluster)."""
    torch = ctx.torch
    N, d = X.shape
    nq = U.shape[0]
    K = crow.shape[0] - 1
    out = ctx.empty((nq, n_top), torch.int32)
    _ck(_fn("lshkm_cluster_top_n", X)(ctx.h, _t_ptr(X), _t_ptr(x_mean), N, d, _t_ptr(crow),
                                      _t_ptr(crows) if crows.numel() else None, K, _t_ptr(U), _t_ptr(u_mean), nq,
                                      _t_ptr(ucl), _t_ptr(unk_ptr), _t_ptr(unk_idx) if unk_idx.numel() else None,
                                      n_top, _t_ptr(out)))
    return out


def cluster_sims(ctx, X, crow, crows, U, ucl, unk_ptr):
    """Sharded clustering recommender, phase 1 (lshkm_cluster_sims): every user's
    similarities to this shard's members of its cluster. Returns (soff [nq+1]
    int64, sims fp64) device tensors."""
    torch = ctx.torch
    N, d = X.shape
    nq = U.shape[0]
    K = crow.shape[0] - 1
    soff = ctx.empty((nq + 1,), torch.int64)
    total = C.c_int64()
    fn = _fn("lshkm_cluster_sims", X)
    cr = _t_ptr(crows) if crows.numel() else None
    _ck(fn(ctx.h, _t_ptr(X), N, d, _t_ptr(crow), cr, K, _t_ptr(U), nq, _t_ptr(ucl), _t_ptr(unk_ptr), _t_ptr(soff),
           None, 0, C.byref(total)))
    sims = ctx.empty((max(total.value, 1),), torch.float64)
    _ck(fn(ctx.h, _t_ptr(X), N, d, _t_ptr(crow), cr, K, _t_ptr(U), nq, _t_ptr(ucl), _t_ptr(unk_ptr), _t_ptr(soff),
           _t_ptr(sims), total.value, C.byref(total)))
    return soff, sims


def cluster_chain(ctx, X, x_mean, crow, crows, ucl, u_mean, unk_ptr, unk_idx, soff, sims, carry=None, n_top=None,
                  carry_out=None):
    """Sharded clustering recommender, phase 2 (lshkm_cluster_chain): the
    prediction sums over this shard's members continued from `carry` (main, abs,
    cnt) or None on the first shard. n_top None: returns the running sums
    (main [total unknowns], abs [nq], cnt [nq]; into carry_out when given);
    else the final [nq][n_top] int32 recommendations."""
    torch = ctx.torch
    N, d = X.shape
    nq = ucl.shape[0]
    K = crow.shape[0] - 1
    M = unk_idx.shape[0]
    cm, ca, cc = carry if carry is not None else (None, None, None)
    out = outs = None
    if n_top is None:
        outs = carry_out if carry_out is not None else (ctx.empty((max(M, 1),), torch.float64),
                                                        ctx.empty((nq,), torch.float64), ctx.empty((nq,), torch.int64))
    else:
        out = ctx.empty((nq, n_top), torch.int32)
    om, oa, oc = outs if outs is not None else (None, None, None)
    _ck(_fn("lshkm_cluster_chain", X)(ctx.h, _t_ptr(X), _t_ptr(x_mean), N, d, _t_ptr(crow),
                                      _t_ptr(crows) if crows.numel() else None, K, nq, _t_ptr(ucl), _t_ptr(u_mean),
                                      _t_ptr(unk_ptr), _t_ptr(unk_idx) if M else None, _t_ptr(soff), _t_ptr(sims),
                                      _t_ptr(cm), _t_ptr(ca), _t_ptr(cc), _t_ptr(om), _t_ptr(oa), _t_ptr(oc),
                                      0 if n_top is None else n_top, _t_ptr(out)))
    return outs if n_top is None else out


def cluster_terms(ctx, X, x_mean, crow, crows, U, ucl, unk_ptr, unk_idx):
    """Sharded clustering recommender, phase 1 in the terms form
    (lshkm_cluster_terms): every user's similarities to this shard's members of
    its cluster and its get_predicted_user_sim terms. Returns (soff, toff, sims,
    terms) device tensors."""
    torch = ctx.torch
    N, d = X.shape
    nq = U.shape[0]
    K = crow.shape[0] - 1
    soff = ctx.empty((nq + 1,), torch.int64)
    toff = ctx.empty((nq + 1,), torch.int64)
    total, tt = C.c_int64(), C.c_int64()
    fn = _fn("lshkm_cluster_terms", X)
    cr = _t_ptr(crows) if crows.numel() else None
    ui = _t_ptr(unk_idx) if unk_idx.numel() else None
    args = (ctx.h, _t_ptr(X), _t_ptr(x_mean), N, d, _t_ptr(crow), cr, K, _t_ptr(U), nq, _t_ptr(ucl), _t_ptr(unk_ptr),
            ui, _t_ptr(soff), _t_ptr(toff))
    # one call when buffers of the previous call's sizes (+1/8) hold this call's
    # output: the library computes only when both totals fit and reports them
    # either way; else a second call into buffers of the reported sizes
    cache = ctx.__dict__.setdefault("_terms_sizes", {})
    key = (str(X.device), X.dtype, nq)
    if key in cache:
        cs, ct = cache[key]
        sims = ctx.empty((cs + cs // 8 + 1,), torch.float64)
        terms = ctx.empty((ct + ct // 8 + 1,), torch.float64)
        _ck(fn(*args, _t_ptr(sims), _t_ptr(terms), sims.numel(), terms.numel(), C.byref(total), C.byref(tt)))
        if total.value <= sims.numel() and tt.value <= terms.numel():
            cache[key] = (total.value, tt.value)
            return soff, toff, sims[:max(total.value, 1)], terms[:max(tt.value, 1)]
    else:
        _ck(fn(*args, None, None, 0, 0, C.byref(total), C.byref(tt)))
    sims = ctx.empty((max(total.value, 1),), torch.float64)
    terms = ctx.empty((max(tt.value, 1),), torch.float64)
    _ck(fn(*args, _t_ptr(sims), _t_ptr(terms), total.value, tt.value, C.byref(total), C.byref(tt)))
    cache[key] = (total.value, tt.value)
    return soff, toff, sims, terms


def cluster_chain_terms(ctx, u_mean, unk_ptr, unk_idx, soff, toff, sims, terms, carry=None, n_top=None):
    """Sharded clustering recommender, phase 2 in the terms form
    (lshkm_cluster_chain_terms): as cluster_chain, from cluster_terms' output."""
    torch = ctx.torch
    nq = u_mean.shape[0]
    M = unk_idx.shape[0]
    cm, ca, cc = carry if carry is not None else (None, None, None)
    out = outs = None
    if n_top is None:
        outs = (ctx.empty((max(M, 1),), torch.float64), ctx.empty((nq,), torch.float64), ctx.empty((nq,), torch.int64))
    else:
        out = ctx.empty((nq, n_top), torch.int32)
    om, oa, oc = outs if outs is not None else (None, None, None)
    _ck(lib().lshkm_cluster_chain_terms(ctx.h, nq, _t_ptr(u_mean), _t_ptr(unk_ptr), _t_ptr(unk_idx) if M else None,
                                        _t_ptr(soff), _t_ptr(toff), _t_ptr(sims), _t_ptr(terms), _t_ptr(cm),
                                        _t_ptr(ca), _t_ptr(cc), _t_ptr(om), _t_ptr(oa), _t_ptr(oc),
                                        0 if n_top is None else n_top, _t_ptr(out)))
    return outs if n_top is None else out


# ------------------------------------------------- reference-named mirrors
def create_LSH_hashtables(ctx, X, metric_type, k, L, lsh_bucket_div, euclidean_h_w, seed):
    """create_LSH_hashtables (lsh_cube.hpp:44-74) with an explicit seed in place of the clock."""
    d = X.shape[1]
    if metric_type == "euclidean":
        V, t, r, _ = params_lsh_euclidean(seed, L, k, d, euclidean_h_w)
        lsh = LSH(ctx, EUCLIDEAN, d, k, L, X.shape[0] // lsh_bucket_div, euclidean_h_w, V=V, t=t, r=r)
    else:
        R, _ = params_lsh_cosine(seed, L, k, d)
        lsh = LSH(ctx, COSINE, d, k, L, R=R)
    lsh.build(X)
    return lsh


def get_LSH_filtered_combined_buckets(lsh, Q, alias_rows=None):
    return lsh.query(Q, True, alias_rows)


def get_LSH_combined_buckets(lsh, Q, alias_rows=None):
    return lsh.query(Q, False, alias_rows)


def create_hypercube(ctx, X, metric_type, k, euclidean_h_w, seed):
    """create_hypercube (lsh_cube.hpp:108-136) with an explicit seed."""
    d = X.shape[1]
    if metric_type == "euclidean":
        V, t, st = params_cube_euclidean(seed, k, d, euclidean_h_w)
        cube = Cube(ctx, EUCLIDEAN, d, k, euclidean_h_w, V=V, t=t, rng_state=st)
    else:
        R, st = params_cube_cosine(seed, k, d)
        cube = Cube(ctx, COSINE, d, k, R=R, rng_state=st)
    cube.build(X)
    return cube


def get_hypercube_combined_buckets(cube, Q, probes):
    return cube.query(Q, probes)


def lloyds_assignment(ctx, X, centroids, metric_type, src_rows=None):
    return lloyd_assign(ctx, X, centroids, metric_type, src_rows)


def k_means(ctx, X, assign, centers, metric_type, min_dist):
    return kmeans_update(ctx, X, assign, centers, metric_type, min_dist)


def k_means_pp(ctx, X, cluster_num, metric_type, seed):
    """k_means_pp with an explicit seed: the chosen rows (centroids[i] = X[rows[i]])."""
    return kmeans_pp_rows(ctx, X, cluster_num, metric_type, seed)


def rand_selection(N, cluster_num, seed):
    return rand_selection_rows(N, cluster_num, seed)
