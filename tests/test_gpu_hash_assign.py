"""GPU parity: projection hashes (LSH euclidean / cosine) and Lloyd assignment
against the reference's golden outputs and the CPU oracle. Bit-exact on all
integer outputs and on the fp64 distances."""
import numpy as np
import pytest

import oracle
from amd import lshkm
from conftest import assert_dist, cases, golden, golden_meta, lloyd_input

META = golden_meta()
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return lshkm.Context(0)


def to_dev(ctx, a):
    return ctx.torch.from_numpy(np.ascontiguousarray(a)).to(ctx.dev)


@pytest.mark.parametrize("name", cases("lsh"))
def test_lsh_hash_golden(ctx, name):
    m, g = META[name], golden(name)
    X = to_dev(ctx, oracle.synth(m["data_seed"], m["N"], m["d"]))
    if m["metric"] == "euclidean":
        lsh = lshkm.LSH(ctx, "euclidean", m["d"], m["k"], m["L"], m["nb"], m["w"], V=g["V"], t=g["t"], r=g["r"])
        tu, ph, bu = lsh.hash(X)
        assert np.array_equal(tu.cpu().numpy(), g["tuples"])
    else:
        lsh = lshkm.LSH(ctx, "cosine", m["d"], m["k"], m["L"], R=g["R"])
        _, ph, bu = lsh.hash(X)
    assert np.array_equal(ph.cpu().numpy(), g["phi"])
    assert np.array_equal(bu.cpu().numpy(), g["bucket"])


def test_lsh_hash_large_vs_oracle(ctx):
    # 200k points at the bench shape (d=128, L=5, k=4, w=0.4, nb=N/100); oracle = x87 restatement.
    N, d, L, k = 200_000, 128, 5, 4
    V, t, r, _ = lshkm.params_lsh_euclidean(12345, L, k, d, 0.4)
    X = ctx.synth(0x5EED, N, d)
    lsh = lshkm.LSH(ctx, "euclidean", d, k, L, N // 100, 0.4, V=V, t=t, r=r)
    tu, ph, bu = lsh.hash(X)
    xt, xp, xb = oracle.lsh_hash_euclid(X.cpu().numpy(), V, t, np.float32(0.4), r, N // 100)
    assert np.array_equal(tu.cpu().numpy(), xt)
    assert np.array_equal(ph.cpu().numpy(), xp)
    assert np.array_equal(bu.cpu().numpy(), xb)


def _near_boundary_points(V, t, w, n, rng):
    """Rows whose (v0.x + t)/w sits within ~1e-15 of an integer: forces the exact path."""
    d = V.shape[-1]
    v = V.reshape(-1, d)[0].astype(np.float64)
    rows = []
    for i in range(n):
        x = np.zeros(d, np.float32)
        target = float(rng.integers(-20, 20))
        x[0] = np.float32((target * w - t.reshape(-1)[0]) / v[0])
        res = (v[0] * np.float64(x[0]) + np.float64(t.reshape(-1)[0])) / w - target
        x[1] = np.float32(-res * w / v[1])
        res2 = (v[0] * np.float64(x[0]) + v[1] * np.float64(x[1]) + np.float64(t.reshape(-1)[0])) / w - target
        x[2] = np.float32(-res2 * w / v[2])
        rows.append(x)
    return np.stack(rows)


def test_hash_exact_path_forced(ctx):
    d, L, k = 128, 1, 4
    V, t, r, _ = lshkm.params_lsh_euclidean(99, L, k, d, 0.4)
    X = _near_boundary_points(V, t, np.float32(0.4), 256, np.random.default_rng(0))
    X = np.concatenate([X, np.zeros((8, d), np.float32)])
    ctx.reset_stats()
    lsh = lshkm.LSH(ctx, "euclidean", d, k, L, 7, 0.4, V=V, t=t, r=r)
    tu, ph, bu = lsh.hash(to_dev(ctx, X))
    xt, xp, xb = oracle.lsh_hash_euclid(X, V, t, np.float32(0.4), r, 7)
    assert np.array_equal(tu.cpu().numpy(), xt)
    assert np.array_equal(ph.cpu().numpy(), xp)
    assert ctx.stat(lshkm.STAT_HASH_EXACT) > 0
    # cosine: the zero vector has an exactly-zero inner product (sign test at the boundary)
    R, _ = lshkm.params_lsh_cosine(7, 2, 5, d)
    cl = lshkm.LSH(ctx, "cosine", d, 5, 2, R=R)
    Z = np.zeros((64, d), np.float32); Z[1:, :] = oracle.synth(5, 63, d)
    ctx.reset_stats()
    _, _, cb = cl.hash(to_dev(ctx, Z))
    assert np.array_equal(cb.cpu().numpy(), oracle.lsh_hash_cosine(Z, R))
    assert ctx.stat(lshkm.STAT_HASH_EXACT) >= 2


@pytest.mark.parametrize("name", cases("lloyd"))
def test_lloyd_golden(ctx, name, dist_mode):
    m, g = META[name], golden(name)
    X = to_dev(ctx, lloyd_input(name))
    for it in range(len(g["cont"])):
        Cc = to_dev(ctx, g[f"centers{it}"])
        src = g["src_rows"] if it == 0 else None
        a, dist = lshkm.lloyd_assign(ctx, X, Cc, m["metric"], src)
        assert np.array_equal(a.cpu().numpy(), g[f"assign{it}"]), it
        gd, rd = dist.cpu().numpy(), g[f"dist{it}"]
        if dist_mode == "certified" and m["metric"] == "euclidean":
            # the certified f32 winner distance (conftest.DIST_TOL)
            assert_dist(gd, rd, "certified")
            continue
        # bit for bit, general fp64 centroids after an update included (glibc's
        # pow(x, 2), csrc/gpow2.h); zero rows under cosine: the x86 default NaN
        assert np.array_equal(gd.view(np.uint64), rd.view(np.uint64)), (it, np.nonzero(gd != rd)[0][:8])


def test_lloyd_large_vs_oracle(ctx, dist_mode):
    N, d, K = 100_000, 128, 256
    X = ctx.synth(0x5EED, N, d)
    rows = np.arange(K) * (N // K)
    Cc = X[ctx.torch.from_numpy(rows.astype(np.int64)).to(ctx.dev)].double()
    a, dist = lshkm.lloyd_assign(ctx, X, Cc, "euclidean", rows.astype(np.int32))
    sub = np.random.default_rng(1).choice(N, 3000, replace=False)
    Xs = X.cpu().numpy()
    oa, od = oracle.lloyd_assign(Xs[sub], Cc.cpu().numpy(), "euclidean", None)
    ga, gd = a.cpu().numpy()[sub], dist.cpu().numpy()[sub]
    over = np.isin(sub, rows)               # centroid rows are overridden to (c, 0)
    assert np.array_equal(ga[~over], oa[~over])
    assert_dist(gd[~over], od[~over], dist_mode)
    assert np.all(gd[over] == 0.0)


def test_lloyd_general_fp64_centroids(ctx, dist_mode):
    # centroids that are not fp32 values (after an update): exact mode keeps the
    # reference's chain bit for bit -- every (x_j - c_j) is a general double, so
    # glibc's pow(x, 2) differs from x*x on some of its squares -- certified 2^-20
    N, d, K = 20_000, 128, 64
    X = ctx.synth(3, N, d)
    Cc = X[:K].double() * (1 + 1e-3) + 1e-5
    ctx.reset_stats()
    a, dist = lshkm.lloyd_assign(ctx, X, Cc, "euclidean")
    oa, od = oracle.lloyd_assign(X.cpu().numpy(), Cc.cpu().numpy(), "euclidean", None)
    assert np.array_equal(a.cpu().numpy(), oa)
    assert_dist(dist.cpu().numpy(), od, dist_mode)
    if dist_mode == "exact":
        assert ctx.stat(lshkm.STAT_POW_FIX) > 0.5 * N         # the pow fix-up list ran


def test_lloyd_ties_and_duplicates(ctx, dist_mode):
    N, d, K = 5000, 32, 16
    X = ctx.synth(11, N, d)
    rows = np.array([0, 1, 1, 2, 3, 3, 3, 4, 5, 6, 7, 8, 9, 9, 10, 11], np.int32)
    Cc = X[ctx.torch.from_numpy(rows.astype(np.int64)).to(ctx.dev)].double()
    ctx.reset_stats()
    a, dist = lshkm.lloyd_assign(ctx, X, Cc, "euclidean", rows)
    oa, od = oracle.lloyd_assign(X.cpu().numpy(), Cc.cpu().numpy(), "euclidean", rows)
    assert np.array_equal(a.cpu().numpy(), oa)
    assert_dist(dist.cpu().numpy(), od, dist_mode)
    assert ctx.stat(lshkm.STAT_ASSIGN_AMBIG) > 0


@pytest.mark.parametrize("form", ["persistent", "chunked"])
def test_hash_assign_fused_vs_oracle(ctx, sctx, sw, form, monkeypatch, dist_mode):
    # the headline path: one pass over the rows (split-f16 MFMA), at 200k rows
    # (ragged: not a multiple of the 32-row tile); both kernel forms (chunked:
    # forced in the test build)
    M, c = (lshkm, ctx) if form == "persistent" else (sw, sctx)
    if form == "chunked":
        monkeypatch.setenv("LSHKM_FUSED_FORM", "chunked")
    N, d, L, k, K = 200_003, 128, 5, 4, 256
    V, t, r, _ = lshkm.params_lsh_euclidean(12345, L, k, d, 0.4)
    X = ctx.synth(0x5EED, N, d)
    lsh = M.LSH(c, "euclidean", d, k, L, N // 100, 0.4, V=V, t=t, r=r)
    rows = (np.arange(K) * (N // K)).astype(np.int32)
    Cc = X[to_dev(ctx, rows.astype(np.int64))].double()
    c.reset_stats()
    tu, ph, bu, a, dist = M.hash_assign(lsh, X, Cc, rows, tuples=True, phi=True, bucket=True)
    Xh = X.cpu().numpy()
    xt, xp, xb = oracle.lsh_hash_euclid(Xh, V, t, np.float32(0.4), r, N // 100)
    assert np.array_equal(tu.cpu().numpy(), xt)
    assert np.array_equal(ph.cpu().numpy(), xp)
    assert np.array_equal(bu.cpu().numpy(), xb)
    sub = np.random.default_rng(5).choice(N, 2500, replace=False)
    oa, od = oracle.lloyd_assign(Xh[sub], Cc.cpu().numpy(), "euclidean", None)
    over = np.isin(sub, rows)
    ga, gd = a.cpu().numpy()[sub], dist.cpu().numpy()[sub]
    assert np.array_equal(ga[~over], oa[~over])
    assert_dist(gd[~over], od[~over], dist_mode if form == "persistent" else "exact")
    amb = c.stat(lshkm.STAT_ASSIGN_AMBIG)
    assert amb < 0.05 * N, amb          # the bound is certifying the vast majority


@pytest.mark.parametrize("path", ["f32", "exact"])
def test_assign_paths_agree(ctx, sctx, sw, path, monkeypatch, dist_mode):
    N, d, K = 30_000, 128, 64
    X = ctx.synth(21, N, d)
    Cc = X[:K].double() * 1.0001
    a0, d0 = lshkm.lloyd_assign(ctx, X, Cc, "euclidean")
    monkeypatch.setenv("LSHKM_ASSIGN_PATH", path)
    a1, d1 = sw.lloyd_assign(sctx, X, Cc, "euclidean")
    assert np.array_equal(a0.cpu().numpy(), a1.cpu().numpy())
    # the f32-MFMA and exact paths always give the exact-order distance
    assert_dist(d0.cpu().numpy(), d1.cpu().numpy(), dist_mode)


@pytest.mark.parametrize("d,K,case", [(128, 256, "rows"), (100, 64, "rows"), (16, 1, "rows"), (256, 300, "scaled"),
                                      (64, 40, "dups"), (32, 20, "zero_c0"), (32, 20, "zero_c5"),
                                      (48, 30, "special")])
def test_cosine_mfma_vs_exact(ctx, sctx, sw, d, K, case, monkeypatch):
    # cosine Lloyd: the certified f32-MFMA path (-x.c/|c| scores) must agree bit
    # for bit with the exact all-centroid pass and with the oracle (assignment.hpp:52-75)
    N = 20_011
    X = ctx.synth(0xC05 + d, N, d)
    rng = np.random.default_rng(d + K)
    rows = rng.choice(N, K, replace=False).astype(np.int64)
    Cc = X[to_dev(ctx, rows)].double()
    if case == "scaled":
        Cc = Cc * to_dev(ctx, rng.uniform(1e-3, 1e3, (K, 1)))    # |c| spread (cosine ignores it)
    elif case == "dups":
        Cc[1::3] = Cc[0::3][: Cc[1::3].shape[0]] * 2.0          # parallel centroids: exact ties
        X[5::7] = X[5::7] * 0.0                                   # zero rows (NaN everywhere)
    elif case == "zero_c0":
        Cc[0] = 0.0                     # the sentinel takes centroid 0's NaN for every row
    elif case == "zero_c5":
        Cc[5] = 0.0                     # never taken
    elif case == "special":
        X[3, 2] = float("inf"); X[10, 0] = float("nan"); X[20] = 1e-41   # inf / nan / denormal rows
        X[30] = X[30] * 1e19                                              # |x| past the f32 range guard
        Cc[7, 1] = 1e-300; Cc[8] = Cc[8] * 1e-12                          # fp32-underflowing entry, tiny norm
    ctx.reset_stats()
    a0, d0 = lshkm.lloyd_assign(ctx, X, Cc, "cosine")
    amb = ctx.stat(lshkm.STAT_ASSIGN_AMBIG)
    monkeypatch.setenv("LSHKM_ASSIGN_PATH", "exact")
    a1, d1 = sw.lloyd_assign(sctx, X, Cc, "cosine")
    assert np.array_equal(a0.cpu().numpy(), a1.cpu().numpy())
    assert np.array_equal(d0.cpu().numpy().view(np.uint64), d1.cpu().numpy().view(np.uint64))
    sub = np.random.default_rng(7).choice(N, 1500, replace=False)
    oa, od = oracle.lloyd_assign(X.cpu().numpy()[sub], Cc.cpu().numpy(), "cosine", None)
    assert np.array_equal(a0.cpu().numpy()[sub], oa)
    assert np.array_equal(d0.cpu().numpy()[sub].view(np.uint64), od.view(np.uint64))
    if case in ("rows", "scaled"):
        assert amb < 0.05 * N, amb      # the bound certifies the vast majority
    if case == "zero_c0":
        assert amb == N


@pytest.mark.parametrize("N,K,L,k", [(1, 1, 1, 4), (65, 64, 8, 4), (4099, 300, 8, 4), (777, 256, 3, 3),
                                     (2048, 200, 2, 4), (1500, 256, 7, 2)])
def test_hash_assign_shapes(ctx, N, K, L, k, dist_mode):
    # persistent form (K <= 256, k = 4) and the chunked form (K > 256 or k != 4)
    d = 128
    Xh = oracle.synth(31 + N, N, d)
    X = to_dev(ctx, Xh)
    V, t, r, _ = lshkm.params_lsh_euclidean(7 + L, L, k, d, 0.5)
    nb = max(N // 10, 1)
    lsh = lshkm.LSH(ctx, "euclidean", d, k, L, nb, 0.5, V=V, t=t, r=r)
    rng = np.random.default_rng(N)
    Ch = rng.choice(Xh, K, replace=True).astype(np.float64) * 1.001
    tu, ph, bu, a, dist = lshkm.hash_assign(lsh, X, to_dev(ctx, Ch), None, tuples=True, phi=True, bucket=True)
    xt, xp, xb = oracle.lsh_hash_euclid(Xh, V, t, np.float32(0.5), r, nb)
    assert np.array_equal(tu.cpu().numpy(), xt)
    assert np.array_equal(ph.cpu().numpy(), xp)
    assert np.array_equal(bu.cpu().numpy(), xb)
    oa, od = oracle.lloyd_assign(Xh, Ch, "euclidean", None)
    assert np.array_equal(a.cpu().numpy(), oa)
    # centroids are not fp32-valued: glibc's pow(x, 2), bit for bit in exact mode
    assert_dist(dist.cpu().numpy(), od, dist_mode)


@pytest.mark.parametrize("form", ["persistent", "chunked"])
def test_fused_range_guard(ctx, sctx, sw, form, monkeypatch, dist_mode):
    # values beyond the f16 range must never be certified by the split path
    # (in the persistent form every function of such a row goes through the fix-up pass)
    M, c = (lshkm, ctx) if form == "persistent" else (sw, sctx)
    if form == "chunked":
        monkeypatch.setenv("LSHKM_FUSED_FORM", "chunked")
    N, d, K, L, k = 3000, 128, 16, 5, 4
    Xh = oracle.synth(8, N, d)
    Xh[::7, 3] = 1.0e5
    Xh[5, :] = 7.0e4
    X = to_dev(ctx, Xh)
    V, t, r, _ = lshkm.params_lsh_euclidean(3, L, k, d, 4.0)
    lsh = M.LSH(c, "euclidean", d, k, L, 30, 4.0, V=V, t=t, r=r)
    Cc = to_dev(ctx, Xh[:K].astype(np.float64))
    tu, _, bu, a, dist = M.hash_assign(lsh, X, Cc, None)
    xt, _, xb = oracle.lsh_hash_euclid(Xh, V, t, np.float32(4.0), r, 30)
    oa, od = oracle.lloyd_assign(Xh, Xh[:K].astype(np.float64), "euclidean", None)
    assert np.array_equal(tu.cpu().numpy(), xt) and np.array_equal(bu.cpu().numpy(), xb)
    assert np.array_equal(a.cpu().numpy(), oa)
    assert_dist(dist.cpu().numpy(), od, dist_mode if form == "persistent" else "exact")
    # and centroids beyond the range
    Cbig = Cc.clone(); Cbig[2, 0] = 5.0e4
    a2, d2 = M.lloyd_assign(c, X, Cbig, "euclidean")
    oa2, od2 = oracle.lloyd_assign(Xh, Cbig.cpu().numpy(), "euclidean", None)
    assert np.array_equal(a2.cpu().numpy(), oa2)
    assert_dist(d2.cpu().numpy(), od2, dist_mode)


@pytest.mark.parametrize("case", ["ties", "near", "nonfinite"])
def test_pruned_exact_pass(ctx, sctx, sw, case, monkeypatch, dist_mode):
    # the listed-row pass (f32 candidate pruning + exact order on the candidates)
    # against the every-centroid pass and the oracle: duplicate centroids (exact
    # ties, first index must win), near-duplicates (many candidates), and rows
    # beyond the f16 range / non-finite centroids (every centroid evaluated)
    N, d, K = 40_000, 128, 256
    Xh = oracle.synth(77, N, d)
    rng = np.random.default_rng(3)
    Ch = Xh[rng.choice(N, K, replace=False)].astype(np.float64)
    if case == "ties":
        Ch[1::2] = Ch[0::2]                       # every centroid duplicated
    elif case == "near":
        Ch[100:164] = Ch[99] * (1.0 + 1e-7 * np.arange(1, 65)[:, None])
    else:
        Xh[::11, 5] = 4.0e4                       # f16 range guard: rows listed
        Ch[7, 3] = np.inf
    X = to_dev(ctx, Xh)
    C = to_dev(ctx, Ch)
    ctx.reset_stats()
    a, dist = lshkm.lloyd_assign(ctx, X, C, "euclidean")
    assert ctx.stat(lshkm.STAT_ASSIGN_AMBIG) > 0
    monkeypatch.setenv("LSHKM_EXACT_PASS", "full")
    a1, d1 = sw.lloyd_assign(sctx, X, C, "euclidean")
    assert np.array_equal(a.cpu().numpy(), a1.cpu().numpy())
    assert np.array_equal(dist.cpu().numpy().view(np.uint64), d1.cpu().numpy().view(np.uint64))
    sub = np.random.default_rng(4).choice(N, 3000, replace=False)
    oa, od = oracle.lloyd_assign(Xh[sub], Ch, "euclidean", None)
    assert np.array_equal(a.cpu().numpy()[sub], oa)
    assert_dist(dist.cpu().numpy()[sub], od, dist_mode)     # "near": non-fp32 centroids, bit for bit


@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("case", ["near_parallel", "near_orthogonal", "cancelling"])
def test_cosine_certified_quotient_adversarial(ctx, sctx, sw, case, d, monkeypatch):
    # exact.h IpAcc: the double-double inner product with the bounded x87
    # rounding must give the soft-x87 bits or decline; every row is checked
    # against the oracle (real long double) on both assignment paths (d = 128:
    # the split-f16 persistent kernel with normalised centroids)
    N, K = 3001, 12
    rng = np.random.default_rng(11)
    Xh = ctx.synth(0xADD, N, d).cpu().numpy().astype(np.float64)
    if case == "near_parallel":          # q = 1 - O(2^-20): 1 - q keeps few bits
        base = Xh[rng.choice(N, K, replace=False)]
        Ch = base * (1.0 + rng.uniform(-2.0**-20, 2.0**-20, base.shape))
        Xh[:K * 50] = np.repeat(base, 50, axis=0).astype(np.float32)
    elif case == "near_orthogonal":      # x.c ~ 0: |S| << sum|S_k|
        Ch = rng.standard_normal((K, d))
        for i in range(K):
            v = Xh[i * 7]
            Ch[i] -= v * (Ch[i] @ v) / (v @ v)
    else:                                # large terms that cancel
        Ch = rng.standard_normal((K, d))
        Ch[:, 0] = 1e8
        Ch[:, 1] = -1e8
        Xh[:, 1] = Xh[:, 0]
    X = to_dev(ctx, Xh.astype(np.float32))
    Cc = to_dev(ctx, np.ascontiguousarray(Ch))
    a0, d0 = lshkm.lloyd_assign(ctx, X, Cc, "cosine")
    monkeypatch.setenv("LSHKM_ASSIGN_PATH", "exact")
    a1, d1 = sw.lloyd_assign(sctx, X, Cc, "cosine")
    oa, od = oracle.lloyd_assign(X.cpu().numpy(), Ch, "cosine", None)
    for a, dd in ((a0, d0), (a1, d1)):
        assert np.array_equal(a.cpu().numpy(), oa)
        assert np.array_equal(dd.cpu().numpy().view(np.uint64), od.view(np.uint64))


@pytest.mark.parametrize("metric", ["euclidean", "cosine"])
def test_multipass_persistent_k1024(ctx, sctx, sw, metric, monkeypatch, dist_mode):
    # K > 256 on the persistent form: one launch per 256-centroid slice with the
    # per-lane (best, runner-up, tile) carried across launches; duplicates in
    # different slices (exact ties: the first index must win) and a ragged last
    # slice (K = 1000 -> 4 launches, the last of 232 rows)
    N, d, K = 20_011, 128, 1000
    X = ctx.synth(0x1024, N, d)
    rng = np.random.default_rng(9)
    rows = rng.choice(N, K, replace=False).astype(np.int64)
    Cc = X[to_dev(ctx, rows)].double()
    Cc[600:610] = Cc[100:110]                         # ties across slices
    Cc[900] = Cc[3] * (2.0 if metric == "cosine" else 1.0)
    ctx.reset_stats()
    a0, d0 = lshkm.lloyd_assign(ctx, X, Cc, metric)
    monkeypatch.setenv("LSHKM_ASSIGN_PATH", "exact")
    a1, d1 = sw.lloyd_assign(sctx, X, Cc, metric)
    mode = dist_mode if metric == "euclidean" else "exact"      # cosine distances are exact-order in both
    assert np.array_equal(a0.cpu().numpy(), a1.cpu().numpy())
    assert_dist(d0.cpu().numpy(), d1.cpu().numpy(), mode)
    sub = np.random.default_rng(2).choice(N, 600, replace=False)
    oa, od = oracle.lloyd_assign(X.cpu().numpy()[sub], Cc.cpu().numpy(), metric, None)
    assert np.array_equal(a0.cpu().numpy()[sub], oa)
    assert_dist(d0.cpu().numpy()[sub], od, mode)


@pytest.mark.parametrize("hashed", [False, True])
def test_two_image_k1000(ctx, sctx, sw, hashed, monkeypatch, dist_mode):
    # the opt-in one-launch form for 512 < K <= 1024 (LSHKM_HI_TWO_IMAGE=1): the
    # block swaps 512-centroid images between the halves of each tile; ties
    # across the images, a ragged second image (K = 1000) and a partial last
    # round, bit-equal to the two-pass default (hash outputs too)
    N, d, K, L, k = 40_011, 128, 1000, 5, 4
    X = ctx.synth(0x21A6, N, d)
    rng = np.random.default_rng(21)
    rows = rng.choice(N, K, replace=False).astype(np.int64)
    Cc = X[to_dev(ctx, rows)].double()
    Cc[700:710] = Cc[100:110]                         # exact ties across the two images
    V, t, r, _ = lshkm.params_lsh_euclidean(77, L, k, d, 0.4)

    def run(M, c):
        if hashed:
            lsh = M.LSH(c, "euclidean", d, k, L, N // 100, 0.4, V=V, t=t, r=r)
            return M.hash_assign(lsh, X, Cc, tuples=True, bucket=True)
        return M.lloyd_assign(c, X, Cc, "euclidean")
    ref = [v.cpu().numpy() for v in run(lshkm, ctx) if v is not None]
    monkeypatch.setenv("LSHKM_HI_TWO_IMAGE", "1")
    got = [v.cpu().numpy() for v in run(sw, sctx) if v is not None]
    assert len(ref) == len(got)
    for a, b in zip(ref[:-1], got[:-1]):                 # tuples / buckets / cluster IDs
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
    assert_dist(got[-1], ref[-1], dist_mode, both_certified=True)


@pytest.mark.parametrize("N,K,case", [(200_000, 256, "rows"), (50_000, 1000, "rows"), (30_011, 64, "special"),
                                      (40_000, 200, "scaled")])
def test_cosine_hash_assign_fused(ctx, N, K, case):
    # main.cpp's cosine flow in one pass (lshkm_hash_assign_metric): CosineGGen
    # buckets and cosine Lloyd from the hi-only kernel with the hash tile, against
    # the two separate calls and the oracle
    d, L, k = 128, 5, 4
    Xh = oracle.synth(0xC0 + K, N, d).copy()
    rng = np.random.default_rng(K)
    if case == "special":
        Xh[5] = 0.0                                   # zero row: NaN distances, bits of exact zeros
        Xh[9] *= np.float32(4e4)                      # beyond the f16 range guard
        Xh[11, :] = np.round(Xh[11, :] * 4) / 4
    X = to_dev(ctx, Xh)
    R, _ = lshkm.params_lsh_cosine(21, L, k, d)
    lsh = lshkm.LSH(ctx, "cosine", d, k, L, R=R)
    Ch = Xh[rng.choice(N, K, replace=False)].astype(np.float64)
    if case == "scaled":
        Ch *= rng.uniform(1e-3, 1e3, (K, 1))
    C = to_dev(ctx, Ch)
    ctx.reset_stats()
    _, ph, bu, a, dist = lshkm.hash_assign(lsh, X, C, phi=True, bucket=True, metric="cosine")
    _, ph2, bu2 = lsh.hash(X, tuples=False)
    a2, d2 = lshkm.lloyd_assign(ctx, X, C, "cosine")
    assert np.array_equal(ph.cpu().numpy(), ph2.cpu().numpy())
    assert np.array_equal(bu.cpu().numpy(), bu2.cpu().numpy())
    assert np.array_equal(a.cpu().numpy(), a2.cpu().numpy())
    assert np.array_equal(dist.cpu().numpy().view(np.uint64), d2.cpu().numpy().view(np.uint64))
    sub = np.random.default_rng(1).choice(N, 1200, replace=False)
    sub = np.union1d(sub, [5, 9, 11]) if case == "special" else sub
    og = oracle.lsh_hash_cosine(Xh[sub], R.reshape(L, k, d))
    assert np.array_equal(bu.cpu().numpy()[sub], og)
    oa, od = oracle.lloyd_assign(Xh[sub], Ch, "cosine", None)
    assert np.array_equal(a.cpu().numpy()[sub], oa)
    assert np.array_equal(dist.cpu().numpy()[sub].view(np.uint64), od.view(np.uint64))


@pytest.mark.parametrize("name", [n for n in cases("lsh") if "_c" in n])
def test_cosine_hash_assign_golden(ctx, name):
    # golden lsh_c* (the reference's CosineGGen buckets) through the fused cosine pass
    m, g = META[name], golden(name)
    Xh = oracle.synth(m["data_seed"], m["N"], m["d"])
    X = to_dev(ctx, Xh)
    lsh = lshkm.LSH(ctx, "cosine", m["d"], m["k"], m["L"], R=g["R"])
    K = min(16, m["N"])
    Ch = Xh[:K].astype(np.float64)
    _, _, bu, a, dist = lshkm.hash_assign(lsh, X, to_dev(ctx, Ch), bucket=True, metric="cosine")
    assert np.array_equal(bu.cpu().numpy(), g["bucket"])
    oa, od = oracle.lloyd_assign(Xh, Ch, "cosine", None)
    assert np.array_equal(a.cpu().numpy(), oa)
    assert np.array_equal(dist.cpu().numpy().view(np.uint64), od.view(np.uint64))


def test_override_rows_change_between_calls(ctx, dist_mode):
    # the override rows are cached on the device while unchanged (api.cpp): a
    # call with other rows (same K) must override those, and a repeat the first
    N, d, K = 20_000, 128, 64
    X = ctx.synth(0x0F0, N, d)
    ra = (np.arange(K) * 300).astype(np.int32)
    rb = ra + 7
    Cc = X[ctx.torch.from_numpy(ra.astype(np.int64)).to(ctx.dev)].double()
    for src in (ra, rb, rb.copy(), ra):
        a, dist = lshkm.lloyd_assign(ctx, X, Cc, "euclidean", src)
        oa, od = oracle.lloyd_assign(X.cpu().numpy(), Cc.cpu().numpy(), "euclidean", src)
        assert np.array_equal(a.cpu().numpy(), oa)
        assert_dist(dist.cpu().numpy(), od, dist_mode)
