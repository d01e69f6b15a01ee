"""GPU parity of the split-f16 MFMA hash (csrc/hash_mfma.hip) against the fp64
hash kernel (LSHKM_HASH_PATH=fp64, csrc/hash.hip) and the CPU oracle: every
family (LSH euclidean tuples/phi/bucket, LSH cosine g, the euclidean cube's h
values / coins / vertices, the cosine cube's vertex), on N(0,1) rows and on
rows built to defeat the certificate (tiny w: most floors listed; zero, tiny,
huge, out-of-f16-range, subnormal and non-finite rows; grid-valued rows with
exact products). Bit-exact throughout."""
import os

import numpy as np
import pytest

import oracle
from amd import lshkm

pytestmark = pytest.mark.gpu
D = 128


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return lshkm.Context(0)


def to_dev(ctx, a):
    return ctx.torch.from_numpy(np.ascontiguousarray(a)).to(ctx.dev)


def rows(n, seed, special=True):
    X = oracle.synth(seed, n, D).copy()
    if special:
        rng = np.random.default_rng(seed)
        X[0] = 0.0
        X[1] *= np.float32(1e-30)
        X[2] *= np.float32(4e4)                    # |x| > 2^15: never certified
        X[3, 5] = np.inf
        X[4, 7] = np.nan
        X[5] = np.float32(2.0 ** -140)             # subnormal rows
        X[6, :] = np.float32(3e38)                 # overflowing products
        X[7:400] = np.round(X[7:400] * 8) / 8      # exact, often tied, sums
        X[400:600] *= np.float32(1e3)
        X[600:700] = rng.integers(-3, 4, (100, D)).astype(np.float32)
    return np.ascontiguousarray(X, np.float32)


class fp64_path:
    """The fp64 hash kernel forced in the test build (LSHKM_HASH_PATH=fp64)."""
    def __enter__(self):
        self.old = os.environ.get("LSHKM_HASH_PATH")
        os.environ["LSHKM_HASH_PATH"] = "fp64"

    def __exit__(self, *a):
        if self.old is None:
            del os.environ["LSHKM_HASH_PATH"]
        else:
            os.environ["LSHKM_HASH_PATH"] = self.old


def host(t):
    return None if t is None else t.cpu().numpy()


@pytest.mark.parametrize("metric,w,L,k", [("euclidean", 0.4, 5, 4), ("euclidean", 0.01, 5, 4),
                                          ("euclidean", 4.0, 3, 7), ("euclidean", 1.0, 2, 16), ("euclidean", 1.0, 1, 30),
                                          ("cosine", 0.0, 5, 4), ("cosine", 0.0, 4, 8)])
def test_lsh_hash_mfma_vs_fp64_and_oracle(ctx, sctx, sw, metric, w, L, k):
    N = 50_000 + 17                                 # ragged last tile
    Xh = rows(N, 77)
    X = to_dev(ctx, Xh)
    if metric == "euclidean":
        V, t, r, _ = lshkm.params_lsh_euclidean(123, L, k, D, w)
        mk = lambda M, c: M.LSH(c, metric, D, k, L, N // 100, w, V=V, t=t, r=r)
    else:
        R, _ = lshkm.params_lsh_cosine(123, L, k, D)
        mk = lambda M, c: M.LSH(c, metric, D, k, L, R=R)
    ctx.reset_stats()
    a = [host(v) for v in mk(lshkm, ctx).hash(X)]
    with fp64_path():
        b = [host(v) for v in mk(sw, sctx).hash(X)]
    for u, v in zip(a, b):
        assert (u is None) == (v is None)
        if u is not None:
            assert np.array_equal(u, v)
    fin = np.isfinite(Xh).all(axis=1) & (np.abs(Xh).max(axis=1) < 1e30)
    sub = np.nonzero(fin)[0][:4000]
    if metric == "euclidean":
        ot, op, ob = oracle.lsh_hash_euclid(Xh[sub], V.reshape(L, k, D), t.reshape(L, k), np.float32(w),
                                            r.reshape(L, k), N // 100)
        assert np.array_equal(a[0][sub], ot) and np.array_equal(a[1][sub], op) and np.array_equal(a[2][sub], ob)
    else:
        og = oracle.lsh_hash_cosine(Xh[sub], R.reshape(L, k, D))
        assert np.array_equal(a[2][sub], og)


@pytest.mark.parametrize("metric", ["euclidean", "cosine"])
def test_lsh_build_query_mfma_vs_fp64(ctx, sctx, sw, metric):
    N = 200_000
    X = ctx.synth(0x5EED, N, D)
    if metric == "euclidean":
        V, t, r, _ = lshkm.params_lsh_euclidean(9, 5, 4, D, 0.4)
        mk = lambda M, c: M.LSH(c, metric, D, 4, 5, N // 100, 0.4, V=V, t=t, r=r)
    else:
        R, _ = lshkm.params_lsh_cosine(9, 5, 4, D)
        mk = lambda M, c: M.LSH(c, metric, D, 4, 5, R=R)
    Q = to_dev(ctx, rows(3000, 5))
    l1 = mk(lshkm, ctx)
    l1.build(X)
    q1 = l1.query(Q, filtered=metric == "euclidean")
    with fp64_path():
        l2 = mk(sw, sctx)
        l2.build(X)
        q2 = l2.query(Q, filtered=metric == "euclidean")
    for tb in range(5):
        p1, i1 = l1.buckets(tb)
        p2, i2 = l2.buckets(tb)
        assert np.array_equal(p1, p2) and np.array_equal(i1, i2), tb
    assert np.array_equal(q1[0], q2[0]) and np.array_equal(q1[1], q2[1])


@pytest.mark.parametrize("metric,k,w", [("euclidean", 14, 2.0), ("euclidean", 12, 0.05), ("cosine", 14, 0.0)])
def test_cube_mfma_vs_fp64_and_oracle(ctx, sctx, sw, metric, k, w):
    N = 300_000
    Xh = rows(N, 31, special=metric == "cosine")
    if metric == "euclidean":                      # the coin memo needs finite, moderate h values
        Xh[:700] = oracle.synth(32, 700, D)
    X = to_dev(ctx, Xh)
    if metric == "euclidean":
        V, t, st = lshkm.params_cube_euclidean(4242, k, D, w)
        mk = lambda M, c: M.Cube(c, metric, D, k, w, V=V, t=t, rng_state=st)
    else:
        R, st = lshkm.params_cube_cosine(4242, k, D)
        mk = lambda M, c: M.Cube(c, metric, D, k, R=R)
    c1 = mk(lshkm, ctx)
    c1.build(X)
    with fp64_path():
        c2 = mk(sw, sctx)
        c2.build(X)
    p1, i1 = c1.buckets()
    p2, i2 = c2.buckets()
    assert np.array_equal(p1, p2) and np.array_equal(i1, i2)
    if metric == "euclidean":
        m1, m2 = c1.memo(), c2.memo()
        for u, v in zip(m1[:3], m2[:3]):
            assert np.array_equal(np.sort(u), np.sort(v))
        assert m1[3] == m2[3]
        memo = oracle.CoinMemo(k, st)
        ov, _ = memo.apply(oracle.cube_h(Xh, V, t, np.float32(w)))
    else:
        ov = oracle.cube_cosine(Xh, R)
    orp, oidx = oracle.bucket_csr(ov[:, None], 1 << k)
    assert np.array_equal(p1, orp[0]) and np.array_equal(i1, oidx[0])


def test_hash_mfma_fixup_counts(ctx, sctx, sw):
    # tiny w lists most rows for the fix-up pass; the soft-x87 path runs on the
    # rows whose fp64 bound cannot decide either (exact ties on grid rows)
    N = 20_000
    Xh = rows(N, 3)
    V, t, r, _ = lshkm.params_lsh_euclidean(1, 5, 4, D, 0.001)
    lsh = lshkm.LSH(ctx, "euclidean", D, 4, 5, 1000, 0.001, V=V, t=t, r=r)
    a = [host(v) for v in lsh.hash(to_dev(ctx, Xh))]
    with fp64_path():
        lsh2 = sw.LSH(sctx, "euclidean", D, 4, 5, 1000, 0.001, V=V, t=t, r=r)
        b = [host(v) for v in lsh2.hash(to_dev(ctx, Xh))]
    for u, v in zip(a, b):
        assert np.array_equal(u, v)
