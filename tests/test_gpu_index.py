"""GPU parity: bucket scatter (CSR), LSH queries, hypercube (vertices, F coins,
probe queries) and the k-means update, against the reference's golden outputs
and the CPU oracle. Everything here is bit-exact."""
import numpy as np
import pytest

import oracle
from amd import lshkm
from conftest import cases, golden, golden_meta, lloyd_input

META = golden_meta()
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return lshkm.Context(0)


def to_dev(ctx, a):
    return ctx.torch.from_numpy(np.ascontiguousarray(a)).to(ctx.dev)


def split_csr(ptr, idx):
    return [idx[ptr[i]:ptr[i + 1]] for i in range(len(ptr) - 1)]


def make_lsh(ctx, m, g):
    if m["metric"] == "euclidean":
        return lshkm.LSH(ctx, "euclidean", m["d"], m["k"], m["L"], m["nb"], m["w"], V=g["V"], t=g["t"], r=g["r"])
    return lshkm.LSH(ctx, "cosine", m["d"], m["k"], m["L"], R=g["R"])


@pytest.mark.parametrize("name", cases("lsh"))
def test_lsh_build_buckets_golden(ctx, name):
    m, g = META[name], golden(name)
    X = to_dev(ctx, oracle.synth(m["data_seed"], m["N"], m["d"]))
    lsh = make_lsh(ctx, m, g)
    lsh.build(X)
    nb, gp, gi = m["nb"], g["members_ptr"], g["members_idx"]
    for l in range(m["L"]):
        rp, idx = lsh.buckets(l)
        assert np.array_equal(rp, gp[l * nb:(l + 1) * nb + 1] - gp[l * nb]), l
        assert np.array_equal(idx, gi[gp[l * nb]:gp[(l + 1) * nb]]), l


@pytest.mark.parametrize("name", cases("lsh"))
def test_lsh_queries_golden(ctx, name):
    m, g = META[name], golden(name)
    X = to_dev(ctx, oracle.synth(m["data_seed"], m["N"], m["d"]))
    Q = np.concatenate([oracle.synth(m["data_seed"], m["N"], m["d"])[:m["nqrows"]],
                        oracle.synth(m["query_seed"], m["Q"], m["d"])])
    lsh = make_lsh(ctx, m, g)
    lsh.build(X)
    # dataset rows carry their own IDs: alias them (first-write-wins map)
    alias = np.full(Q.shape[0], -1, np.int32); alias[:m["nqrows"]] = np.arange(m["nqrows"])
    for kind, filt in (("qfilt", True), ("qunf", False)):
        ptr, idx = lsh.query(to_dev(ctx, Q), filtered=filt, alias_rows=to_dev(ctx, alias))
        assert np.array_equal(ptr, g[kind + "_ptr"]), kind
        assert np.array_equal(idx, g[kind + "_idx"]), kind


def test_lsh_build_and_query_large_vs_oracle(ctx):
    # C2 shape: 1M x 128, L=5, k=4, w=0.4, nb = N/100 = 10,000
    N, d, L, k = 1_000_000, 128, 5, 4
    V, t, r, _ = lshkm.params_lsh_euclidean(12345, L, k, d, 0.4)
    X = ctx.synth(0x5EED, N, d)
    lsh = lshkm.LSH(ctx, "euclidean", d, k, L, N // 100, 0.4, V=V, t=t, r=r)
    lsh.build(X)
    Xh = X.cpu().numpy()
    tu, _, b = oracle.lsh_hash_euclid(Xh, V, t, np.float32(0.4), r, N // 100)
    orp, oidx = oracle.bucket_csr(b, N // 100)
    for l in range(L):
        rp, idx = lsh.buckets(l)
        assert np.array_equal(rp, orp[l]) and np.array_equal(idx, oidx[l]), l
    qrows = np.random.default_rng(7).choice(N, 500, replace=False).astype(np.int32)
    ptr, out = lsh.query(X[to_dev(ctx, qrows.astype(np.int64))], True, to_dev(ctx, qrows))
    for q, row in enumerate(qrows):
        exp = oracle.lsh_query(N, N // 100, orp, oidx, b[row], tu, tu[row])
        assert np.array_equal(out[ptr[q]:ptr[q + 1]], exp), q
        assert row in exp


def test_lsh_query_empty_and_unbuilt(ctx):
    m, g = META["lsh_e"], golden("lsh_e")
    lsh = make_lsh(ctx, m, g)
    with pytest.raises(lshkm.LshkmError):
        lsh.query(ctx.synth(1, 4, m["d"]))
    lsh.build(to_dev(ctx, oracle.synth(m["data_seed"], m["N"], m["d"])))
    ptr, idx = lsh.query(ctx.synth(1, 0, m["d"]))
    assert ptr.tolist() == [0] and idx.size == 0


@pytest.mark.parametrize("name", cases("cube"))
def test_cube_golden(ctx, name):
    m, g = META[name], golden(name)
    Xh = oracle.synth(m["data_seed"], m["N"], m["d"])
    X = to_dev(ctx, Xh)
    k = m["k"]
    if m["metric"] == "euclidean":
        V, t, st = lshkm.params_cube_euclidean(m["seed"], k, m["d"], m["w"])
        assert np.array_equal(V, g["V"]) and np.array_equal(t, g["t"])
        cube = lshkm.Cube(ctx, "euclidean", m["d"], k, m["w"], V=V, t=t, rng_state=st)
    else:
        R, st = lshkm.params_cube_cosine(m["seed"], k, m["d"])
        cube = lshkm.Cube(ctx, "cosine", m["d"], k, R=R, rng_state=st)
    cube.build(X)
    rp, idx = cube.buckets()
    assert np.array_equal(rp, g["members_ptr"]) and np.array_equal(idx, g["members_idx"])
    assert np.array_equal(cube.vertices(X).cpu().numpy(), g["vertex"])
    if m["metric"] == "euclidean":
        f, h, b, _ = cube.memo()
        o = np.lexsort((h, f))
        assert np.array_equal(f[o], g["memo_f"]) and np.array_equal(h[o], g["memo_h"])
        assert np.array_equal(b[o], g["memo_bit"])
    Q = np.concatenate([Xh[:m["nqrows"]], oracle.synth(m["query_seed"], m["Q"], m["d"])])[g["qmask"].astype(bool)]
    for p in m["probes"]:
        ptr, out = cube.query(to_dev(ctx, Q), p)
        assert np.array_equal(ptr, g[f"q_probes{p}_ptr"]), p
        assert np.array_equal(out, g[f"q_probes{p}_idx"]), p


def test_cube_large_and_continued_coins_vs_oracle(ctx):
    # C4 shape at 1M: d'=14 euclidean; then external queries continue the coin stream
    N, d, k, w = 1_000_000, 128, 14, 2.0
    V, t, st = lshkm.params_cube_euclidean(4242, k, d, w)
    X = ctx.synth(0x5EED, N, d)
    cube = lshkm.Cube(ctx, "euclidean", d, k, w, V=V, t=t, rng_state=st)
    cube.build(X)
    Xh = X.cpu().numpy()
    memo = oracle.CoinMemo(k, st)
    ov, draws = memo.apply(oracle.cube_h(Xh, V, t, np.float32(w)))
    rp, idx = cube.buckets()
    orp, oidx = oracle.bucket_csr(ov[:, None], 1 << k)
    assert np.array_equal(rp, orp[0]) and np.array_equal(idx, oidx[0])
    # far-away queries hit unseen h values: new coins, drawn in (query, f) order
    Qh = (oracle.synth(99, 2000, d) * 6.0).astype(np.float32)
    qv = cube.vertices(to_dev(ctx, Qh)).cpu().numpy()
    oq, nd = memo.apply(oracle.cube_h(Qh, V, t, np.float32(w)))
    assert nd > 0
    assert np.array_equal(qv, oq)
    f, h, b, st_gpu = cube.memo()
    of, oh, ob = memo.as_lists()
    o1, o2 = np.lexsort((h, f)), np.lexsort((oh, of))
    assert np.array_equal(f[o1], of[o2]) and np.array_equal(h[o1], oh[o2]) and np.array_equal(b[o1], ob[o2])
    assert st_gpu == memo.state.value
    ptr, out = cube.query(to_dev(ctx, Xh[:300]), 14)
    for q in range(300):
        seq = oracle.cube_probe_seq(ov[q], 14, k)
        exp = np.concatenate([oidx[0][orp[0][v]:orp[0][v + 1]] for v in seq])
        assert np.array_equal(out[ptr[q]:ptr[q + 1]], exp), q


@pytest.mark.parametrize("k,N", [(7, 5001), (13, 777), (14, 64 * 300 + 63), (3, 1)])
def test_cube_narrow_h_odd_shapes_vs_oracle(ctx, k, N):
    # int16 h with odd k / ragged row counts through the staged row loads
    d, w = 128, 2.0
    V, t, st = lshkm.params_cube_euclidean(k * 31 + N, k, d, w)
    Xh = oracle.synth(N + k, N, d)
    cube = lshkm.Cube(ctx, "euclidean", d, k, w, V=V, t=t, rng_state=st)
    cube.build(to_dev(ctx, Xh))
    memo = oracle.CoinMemo(k, st)
    ov, _ = memo.apply(oracle.cube_h(Xh, V, t, np.float32(w)))
    rp, idx = cube.buckets()
    orp, oidx = oracle.bucket_csr(ov[:, None], 1 << k)
    assert np.array_equal(rp, orp[0]) and np.array_equal(idx, oidx[0])
    assert cube.memo()[3] == memo.state.value


def test_cube_wide_h_range_vs_oracle(ctx):
    # h beyond int16 (w = 1e-4): the narrow h output saturates, the batch is
    # hashed again as int32; vertices, buckets and the coin stream stay exact
    N, d, k, w = 3000, 128, 6, 1e-4
    V, t, st = lshkm.params_cube_euclidean(77, k, d, w)
    Xh = oracle.synth(0xB16, N, d)
    cube = lshkm.Cube(ctx, "euclidean", d, k, w, V=V, t=t, rng_state=st)
    cube.build(to_dev(ctx, Xh))
    hh = oracle.cube_h(Xh, V, t, np.float32(w))
    assert np.abs(hh).max() > 32767
    memo = oracle.CoinMemo(k, st, hmin=int(hh.min()), hspan=int(hh.max() - hh.min()) + 1)
    ov, _ = memo.apply(hh)
    rp, idx = cube.buckets()
    orp, oidx = oracle.bucket_csr(ov[:, None], 1 << k)
    assert np.array_equal(rp, orp[0]) and np.array_equal(idx, oidx[0])
    assert cube.memo()[3] == memo.state.value


def test_cube_sharded_build_matches_single(ctx):
    # shards export unseen (f, h), merge in global first-occurrence
    # order, draw on the host, import, build -> per-shard vertices, memo and
    # engine state equal to one cube over all rows (3 shards, one empty).
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "sharding", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                 "crypto-recommendation_amd", "sharding.py"))
    sharding = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sharding)
    N, d, k, w = 200_000, 128, 14, 2.0
    V, t, st = lshkm.params_cube_euclidean(31337, k, d, w)
    X = ctx.synth(0x5EED, N, d)
    whole = lshkm.Cube(ctx, "euclidean", d, k, w, V=V, t=t, rng_state=st)
    whole.build(X)
    vw = whole.vertices(X).cpu().numpy()
    cuts = [0, 70_000, 70_000, N]
    cubes = [lshkm.Cube(ctx, "euclidean", d, k, w, V=V, t=t, rng_state=st) for _ in cuts[1:]]
    parts = []
    for cb, lo, hi in zip(cubes, cuts, cuts[1:]):
        f, h, r = cb.unseen(X[lo:hi])
        parts.append((f, h, r + lo))
    fs, hs = sharding.merge_unseen(parts, k)
    bits, st2 = lshkm.coins_draw(st, hs)
    wf, wh, wb, wst = whole.memo()
    assert st2 == wst and len(fs) == len(wf)
    for cb, lo, hi in zip(cubes, cuts, cuts[1:]):
        cb.import_coins(fs, hs, bits, st2)
        cb.build(X[lo:hi])
        if hi > lo:
            assert np.array_equal(cb.vertices(X[lo:hi]).cpu().numpy(), vw[lo:hi])
        rp, idx = cb.buckets()
        assert rp[-1] == hi - lo
        f, h, b, s = cb.memo()
        assert s == wst
        o1, o2 = np.lexsort((h, f)), np.lexsort((wh, wf))
        assert np.array_equal(f[o1], wf[o2]) and np.array_equal(h[o1], wh[o2]) and np.array_equal(b[o1], wb[o2])


@pytest.mark.parametrize("name", cases("lloyd"))
def test_kmeans_update_golden(ctx, name):
    m, g = META[name], golden(name)
    X = to_dev(ctx, lloyd_input(name))
    for it in range(len(g["cont"])):
        a = to_dev(ctx, g[f"assign{it}"])
        Cold = to_dev(ctx, g[f"centers{it}"])
        Cn, cnt, cont = lshkm.kmeans_update(ctx, X, a, Cold, m["metric"], m["min_dist"])
        assert cont == bool(g["cont"][it]), it
        exp = g[f"centers{it + 1}"] if cont else oracle.kmeans_update(
            lloyd_input(name), g[f"assign{it}"], g[f"centers{it}"], m["metric"], m["min_dist"])[0]
        assert np.array_equal(Cn.cpu().numpy().view(np.uint64), exp.view(np.uint64)), it
        assert np.array_equal(cnt.cpu().numpy(), np.bincount(g[f"assign{it}"], minlength=m["K"])), it


def test_kmeans_update_large_vs_oracle(ctx):
    N, d, K = 1_000_000, 128, 256
    X = ctx.synth(0x5EED, N, d)
    a = ctx.torch.randint(0, K, (N,), dtype=ctx.torch.int32, device=ctx.dev)
    a[:5] = 3                      # uneven, and one empty cluster
    a[a == 17] = 18
    Cold = ctx.torch.zeros((K, d), dtype=ctx.torch.float64, device=ctx.dev)
    Cn, cnt, cont = lshkm.kmeans_update(ctx, X, a, Cold, "euclidean", 0.05)
    on, ocnt, ocont = oracle.kmeans_update(X.cpu().numpy(), a.cpu().numpy(), Cold.cpu().numpy(), "euclidean", 0.05)
    assert cont == ocont
    assert np.array_equal(cnt.cpu().numpy(), ocnt) and ocnt[17] == 0
    assert np.array_equal(Cn.cpu().numpy().view(np.uint64), on.view(np.uint64))
    # sharded fast mode: per-shard exact-order sums + a sum of partials
    s1, c1 = lshkm.kmeans_partial(ctx, X[:N // 2], a[:N // 2], K)
    s2, c2 = lshkm.kmeans_partial(ctx, X[N // 2:], a[N // 2:], K)
    C2, cont2 = lshkm.kmeans_finalize(ctx, s1 + s2, c1 + c2, Cold, "euclidean", 0.05)
    assert np.array_equal((c1 + c2).cpu().numpy(), ocnt)
    rel = (C2 - Cn).abs().max().item() / Cn.abs().max().item()
    assert rel < 1e-13 and cont2 == cont
    # sharded exact mode: 3 uneven shards (one empty) chained through carries
    cuts = [0, N // 3, N // 3, N]
    cs = cc = None
    for lo, hi in zip(cuts, cuts[1:]):
        cs, cc = lshkm.kmeans_partial_carry(ctx, X[lo:hi], a[lo:hi], K, cs, cc)
    C3, cont3 = lshkm.kmeans_finalize(ctx, cs, cc, Cold, "euclidean", 0.05)
    assert np.array_equal(cc.cpu().numpy(), ocnt) and cont3 == cont
    assert np.array_equal(C3.cpu().numpy().view(np.uint64), on.view(np.uint64))      # bit-exact


def test_queries_large_batches_multiblock_scan(ctx):
    # query batches whose per-slot size arrays exceed one scan block (nq * S and
    # nq * L > 32768): the multi-block scan must give the same CSR as the sizes
    N, d, k = 200_000, 32, 10
    X = ctx.synth(41, N, d)
    Xh = X.cpu().numpy()
    V, t, st = lshkm.params_cube_euclidean(5, k, d, 2.0)
    cube = lshkm.Cube(ctx, "euclidean", d, k, 2.0, V=V, t=t, rng_state=st)
    cube.build(X)
    nq, probes = 40_000, 10
    rows = np.random.default_rng(1).choice(N, nq, replace=False)
    Q = X[to_dev(ctx, rows.astype(np.int64))]
    ptr, idx = cube.query(Q, probes)
    rp, bidx = cube.buckets()
    qv = cube.vertices(Q).cpu().numpy()
    sizes = np.diff(rp)
    want = np.zeros(nq + 1, np.int64)
    seqs = [oracle.cube_probe_seq(int(v), probes, k) for v in qv]
    want[1:] = np.cumsum([sizes[s].sum() for s in seqs])
    assert np.array_equal(ptr, want)
    for q in np.random.default_rng(2).choice(nq, 200, replace=False):
        got = idx[ptr[q]:ptr[q + 1]]
        exp = np.concatenate([bidx[rp[v]:rp[v + 1]] for v in seqs[q]])
        assert np.array_equal(got, exp), q
    # LSH: 30k queries x L = 5 tables
    L, kk = 5, 4
    V2, t2, r2, _ = lshkm.params_lsh_euclidean(9, L, kk, d, 1.0)
    lsh = lshkm.LSH(ctx, "euclidean", d, kk, L, N // 100, 1.0, V=V2, t=t2, r=r2)
    lsh.build(X)
    qr = rows[:30_000]
    ptr2, out2 = lsh.query(Q[:30_000], False)
    _, _, qb = oracle.lsh_hash_euclid(Xh[qr], V2, t2, np.float32(1.0), r2, N // 100)
    _, _, b = oracle.lsh_hash_euclid(Xh, V2, t2, np.float32(1.0), r2, N // 100)
    orp, oidx = oracle.bucket_csr(b, N // 100)
    for q in np.random.default_rng(3).choice(30_000, 100, replace=False):
        exp = oracle.lsh_query(N, N // 100, orp, oidx, qb[q])
        assert np.array_equal(out2[ptr2[q]:ptr2[q + 1]], exp), q


@pytest.mark.parametrize("k,w", [(14, 2.0), (10, 40.0)])
def test_cube_query_load_balanced_copy_full(ctx, k, w):
    # every output element checked (vectorised): k = 14 leaves most slots tiny
    # (a chunk spans many slots, some empty); w = 40 puts
    # most rows in a few huge vertices (slots far larger than a chunk)
    N, d = 200_000, 32
    X = ctx.synth(43, N, d)
    V, t, st = lshkm.params_cube_euclidean(7, k, d, w)
    cube = lshkm.Cube(ctx, "euclidean", d, k, w, V=V, t=t, rng_state=st)
    cube.build(X)
    nq, probes = 20_000, k
    rows = np.random.default_rng(4).choice(N, nq, replace=False)
    Q = X[to_dev(ctx, rows.astype(np.int64))]
    ptr, out = cube.query(Q, probes)
    rp, bidx = cube.buckets()
    qv = cube.vertices(Q).cpu().numpy()
    seqs = np.array([oracle.cube_probe_seq(int(v), probes, k) for v in qv], np.int64)   # [nq, S]
    sz = (rp[seqs + 1] - rp[seqs]).ravel()
    slot_off = np.zeros(sz.size + 1, np.int64)
    slot_off[1:] = np.cumsum(sz)
    assert np.array_equal(ptr, slot_off[::seqs.shape[1]])
    assert sz.max() > 4096 or np.median(sz) < 64            # the regime each case is for
    src = np.repeat(rp[seqs.ravel()] - slot_off[:-1], sz) + np.arange(slot_off[-1], dtype=np.int64)
    assert np.array_equal(out, bidx[src])


def test_lsh_two_phase_reuse_guards(ctx):
    # the filling call reuses the sizing call's state only for the same query
    # batch with nothing in between; interleaved sizing calls must not leak
    import ctypes as C
    N, d, L, k = 50_000, 32, 5, 4
    X = ctx.synth(77, N, d)
    V, t, r, _ = lshkm.params_lsh_euclidean(3, L, k, d, 1.0)
    lsh = lshkm.LSH(ctx, "euclidean", d, k, L, N // 100, 1.0, V=V, t=t, r=r)
    lsh.build(X)
    Q1, Q2 = X[:3000].clone(), X[20_000:24_000].clone()
    want1 = lsh.query(Q1, True)
    lib, p = lshkm.lib(), lshkm._t_ptr
    for q in (Q1, Q2):
        ptr = ctx.empty((q.shape[0] + 1,), ctx.torch.int64)
        tot = C.c_int64()
        lshkm._ck(lib.lshkm_lsh_query(lsh.h, p(q), q.shape[0], None, 1, p(ptr), None, 0, C.byref(tot)))
    # state now belongs to Q2: a fill for Q1 must recompute everything
    ptr1 = ctx.empty((Q1.shape[0] + 1,), ctx.torch.int64)
    out1 = ctx.empty((max(len(want1[1]), 1),), ctx.torch.int32)
    tot = C.c_int64()
    lshkm._ck(lib.lshkm_lsh_query(lsh.h, p(Q1), Q1.shape[0], None, 1, p(ptr1), p(out1), out1.shape[0], C.byref(tot)))
    ctx.sync()
    assert tot.value == len(want1[1])
    assert np.array_equal(ptr1.cpu().numpy(), want1[0]) and np.array_equal(out1.cpu().numpy()[:tot.value], want1[1])
    # a sizing call, then another context user (k-means update scatter), then the fill
    ptr2 = ctx.empty((Q1.shape[0] + 1,), ctx.torch.int64)
    lshkm._ck(lib.lshkm_lsh_query(lsh.h, p(Q1), Q1.shape[0], None, 1, p(ptr2), None, 0, C.byref(tot)))
    lsh2 = lshkm.LSH(ctx, "euclidean", d, k, L, N // 50, 1.0, V=V, t=t, r=r)
    lsh2.build(X)                                       # reuses the context's scatter slots
    lsh2.query(Q2, True)
    out2 = ctx.empty((max(len(want1[1]), 1),), ctx.torch.int32)
    lshkm._ck(lib.lshkm_lsh_query(lsh.h, p(Q1), Q1.shape[0], None, 1, p(ptr2), p(out2), out2.shape[0], C.byref(tot)))
    ctx.sync()
    assert np.array_equal(ptr2.cpu().numpy(), want1[0]) and np.array_equal(out2.cpu().numpy()[:tot.value], want1[1])
    # sizing into one offsets buffer, filling with a fresh one (poisoned): the
    # fill must not trust the reuse state and must write the fresh out_ptr itself
    ptr3 = ctx.empty((Q1.shape[0] + 1,), ctx.torch.int64)
    lshkm._ck(lib.lshkm_lsh_query(lsh.h, p(Q1), Q1.shape[0], None, 1, p(ptr3), None, 0, C.byref(tot)))
    ptr4 = ctx.empty((Q1.shape[0] + 1,), ctx.torch.int64)
    ptr4.fill_(-(1 << 40))
    out4 = ctx.empty((max(len(want1[1]), 1),), ctx.torch.int32)
    lshkm._ck(lib.lshkm_lsh_query(lsh.h, p(Q1), Q1.shape[0], None, 1, p(ptr4), p(out4), out4.shape[0], C.byref(tot)))
    ctx.sync()
    assert tot.value == len(want1[1])
    assert np.array_equal(ptr4.cpu().numpy(), want1[0]) and np.array_equal(out4.cpu().numpy()[:tot.value], want1[1])
