"""Pin the CPU oracle (oracle/lshkm_oracle.c) against the reference's own
outputs (tests/golden, made by oracle/_ref/ref_harness from /root/reference).

Everything here is bit-exact: integer outputs by array_equal, fp64 outputs by
bitwise equality. CPU only.
"""
import numpy as np
import pytest

import oracle
from conftest import case_queries, case_rows, cases, golden, golden_meta, kpp_input, lloyd_input

META = golden_meta()
# the same checks over general fp64 rows (fixtures made from user-vector-shaped
# doubles, tests/golden/make_golden.py:user_vectors; inputs stored in the npz)
LSH = cases("lsh") + cases("f64_lsh")
CUBE = cases("cube") + cases("f64_cube")
LLOYD = cases("lloyd") + cases("f64_lloyd")
KPP = cases("kmeanspp") + cases("f64_kmeanspp")
RANGE = cases("range") + cases("f64_range")


@pytest.mark.parametrize("name", LSH)
def test_lsh_params(name):
    m, g = META[name], golden(name)
    if m["metric"] == "euclidean":
        V, t, r, _ = oracle.gen_lsh_euclid(m["seed"], m["L"], m["k"], m["d"], np.float32(m["w"]))
        assert np.array_equal(V, g["V"]) and np.array_equal(t, g["t"]) and np.array_equal(r, g["r"])
        assert np.all(g["w"] == np.float32(m["w"]))
    else:
        R, _ = oracle.gen_lsh_cosine(m["seed"], m["L"], m["k"], m["d"])
        assert np.array_equal(R.view(np.uint64), g["R"].view(np.uint64))


@pytest.mark.parametrize("name", LSH)
def test_lsh_hash_and_buckets(name):
    m, g = META[name], golden(name)
    X = case_rows(name)
    if m["metric"] == "euclidean":
        tu, phi, b = oracle.lsh_hash_euclid(X, g["V"], g["t"], g["w"][0, 0], g["r"], m["nb"])
        assert np.array_equal(tu, g["tuples"])
        assert np.array_equal(phi, g["phi"])
    else:
        b = oracle.lsh_hash_cosine(X, g["R"])
        assert np.array_equal(b, g["phi"])
    assert np.array_equal(b, g["bucket"])
    rp, idx = oracle.bucket_csr(b, m["nb"])
    # golden CSR is the concatenation over tables of nb buckets each
    L, nb = m["L"], m["nb"]
    gp, gi = g["members_ptr"], g["members_idx"]
    for l in range(L):
        assert np.array_equal(rp[l], gp[l * nb:(l + 1) * nb + 1] - gp[l * nb])
        assert np.array_equal(idx[l], gi[gp[l * nb]:gp[(l + 1) * nb]])


@pytest.mark.parametrize("name", LSH)
def test_lsh_queries(name):
    m, g = META[name], golden(name)
    X = case_rows(name)
    Qx = case_queries(name)
    allq = np.concatenate([X[:m["nqrows"]], Qx])
    nb, L = m["nb"], m["L"]
    if m["metric"] == "euclidean":
        tu, _, b = oracle.lsh_hash_euclid(X, g["V"], g["t"], g["w"][0, 0], g["r"], nb)
        qtu, _, qb = oracle.lsh_hash_euclid(allq, g["V"], g["t"], g["w"][0, 0], g["r"], nb)
    else:
        b = oracle.lsh_hash_cosine(X, g["R"]); qb = oracle.lsh_hash_cosine(allq, g["R"])
        tu = qtu = None
    rp, idx = oracle.bucket_csr(b, nb)
    for kind in ("qfilt", "qunf"):
        ptr, gidx = g[kind + "_ptr"], g[kind + "_idx"]
        for q in range(allq.shape[0]):
            filt = kind == "qfilt" and tu is not None
            got = oracle.lsh_query(m["N"], nb, rp, idx, qb[q], tu if filt else None, qtu[q] if filt else None)
            assert np.array_equal(got, gidx[ptr[q]:ptr[q + 1]]), (kind, q)


@pytest.mark.parametrize("name", CUBE)
def test_cube(name):
    m, g = META[name], golden(name)
    X = case_rows(name)
    k = m["k"]
    if m["metric"] == "euclidean":
        V, t, st = oracle.gen_cube_euclid(m["seed"], k, m["d"], np.float32(m["w"]))
        assert np.array_equal(V, g["V"]) and np.array_equal(t, g["t"])
        h = oracle.cube_h(X, V, t, g["w"][0])
        assert np.array_equal(h, g["h"])
        memo = oracle.CoinMemo(k, st)
        vertex, draws = memo.apply(h)
        f, hh, bit = memo.as_lists()
        o = np.lexsort((hh, f))
        assert np.array_equal(f[o], g["memo_f"]) and np.array_equal(hh[o], g["memo_h"])
        assert np.array_equal(bit[o], g["memo_bit"])
        assert draws == len(g["memo_h"])
    else:
        R, _ = oracle.gen_cube_cosine(m["seed"], k, m["d"])
        assert np.array_equal(R.view(np.uint64), g["R"].view(np.uint64))
        vertex = oracle.cube_cosine(X, R)
    assert np.array_equal(vertex, g["vertex"])
    rp, idx = oracle.bucket_csr(vertex[:, None], 1 << k)
    assert np.array_equal(rp[0], g["members_ptr"]) and np.array_equal(idx[0], g["members_idx"])
    # probe queries (only the fully-seen ones are pinned: qmask)
    Qx = case_queries(name)
    allq = np.concatenate([X[:m["nqrows"]], Qx])[g["qmask"].astype(bool)]
    if m["metric"] == "euclidean":
        qv, _ = memo.apply(oracle.cube_h(allq, V, t, g["w"][0]))
        assert memo.as_lists()[0].size == len(g["memo_h"])  # no new draws for seen queries
    else:
        qv = oracle.cube_cosine(allq, R)
    for p in m["probes"]:
        ptr, gi = g[f"q_probes{p}_ptr"], g[f"q_probes{p}_idx"]
        for q in range(allq.shape[0]):
            seq = oracle.cube_probe_seq(qv[q], p, k)
            got = np.concatenate([idx[0][rp[0][v]:rp[0][v + 1]] for v in seq])
            assert np.array_equal(got, gi[ptr[q]:ptr[q + 1]]), (p, q)


@pytest.mark.parametrize("name", LLOYD)
def test_lloyd_and_update(name):
    m, g = META[name], golden(name)
    X = case_rows(name)
    C = g["centers0"]
    src = g["src_rows"]
    if m.get("init") in ("ext", "ext_far"):
        assert np.array_equal(C, g["ext_centers"])
    for it in range(len(g["cont"])):
        a, dist = oracle.lloyd_assign(X, C, m["metric"], src if it == 0 else None)
        assert np.array_equal(a, g[f"assign{it}"]), it
        assert np.array_equal(dist.view(np.uint64), g[f"dist{it}"].view(np.uint64)), it
        Cn, cnt, cont = oracle.kmeans_update(X, a, C, m["metric"], m["min_dist"])
        assert cont == bool(g["cont"][it])
        C = Cn if cont else C
        assert np.array_equal(C.view(np.uint64), g[f"centers{it + 1}"].view(np.uint64)), it


@pytest.mark.parametrize("name", KPP)
def test_kmeans_pp_and_rand_selection(name):
    m, g = META[name], golden(name)
    X = case_rows(name)
    assert np.array_equal(oracle.kmeans_pp(X, m["K"], m["metric"], m["seed"]), g["kpp_rows"])
    assert np.array_equal(oracle.rand_selection(m["N"], m["K"], m["seed"]), g["rand_rows"])


@pytest.mark.parametrize("name", cases("recom"))
def test_recommend_step(name):
    m, g = META[name], golden(name)
    idx, sim, cnt = oracle.p_closest(g["x"], g["u"], g["cand_ptr"], g["cand_idx"], m["P"])
    assert np.array_equal(cnt, g["pc_cnt"])
    assert np.array_equal(idx, g["pc_idx"])
    assert np.array_equal(sim.view(np.uint64), g["pc_sim"].view(np.uint64))
    top = oracle.top_n_recom(g["x"], g["xmean"], g["u"], g["umean"], g["unk_ptr"], g["unk_idx"], idx, sim, cnt,
                             m["NTOP"])
    has = cnt > 0                     # main.cpp:161 skips users without neighbours
    assert np.array_equal(top[has], g["top"][has])


def test_probe_sequence_rules():
    # lsh_cube.hpp:148-150 quirk: probes == 1 skips Hamming distance 1.
    assert list(oracle.cube_probe_seq(0, 1, 4)) == [0, 0b11]
    assert list(oracle.cube_probe_seq(0, 0, 4)) == [0]
    assert list(oracle.cube_probe_seq(0, 2, 4)) == [0, 1, 2]
    # exhausted cube stops (lsh_cube.hpp:171-172): k=2 -> 3 neighbours max
    assert list(oracle.cube_probe_seq(0, 50, 2)) == [0, 1, 2, 3]
    # distance-2 order: (0,1),(0,2),(0,3),(1,2),...
    assert list(oracle.cube_probe_seq(0, 6, 4))[5:] == [0b0011, 0b0101]


def test_minstd_and_uniform_int():
    import ctypes
    s = ctypes.c_uint32(oracle.lib().or_minstd_seed(1))
    # minstd_rand0 from seed 1: 16807, 282475249, ...
    vals = [oracle.lib().or_uniform_int(ctypes.byref(s), 0, 2147483645) for _ in range(2)]
    assert vals == [16806, 282475248]
    assert oracle.lib().or_minstd_seed(0) == 1 and oracle.lib().or_minstd_seed(2147483647) == 1


@pytest.mark.parametrize("name", RANGE)
def test_range_assignment(name):
    # lsh_/cube_range_assignment (assignment.hpp:108-145) on the reference's own
    # combined buckets; iterations >= 1 run on "k_means_center" centroids whose
    # shared ID collapses the distance cache (key = all zeros).
    m, g = META[name], golden(name)
    X = case_rows(name)
    for it in range(int(g["iters"][0])):
        a, dist, _ = oracle.range_assign(X, g[f"centers{it}"], g[f"comb{it}_ptr"], g[f"comb{it}_idx"], m["metric"],
                                         key=g[f"key{it}"], src_rows=g["src_rows"] if it == 0 else None)
        assert np.array_equal(a, g[f"assign{it}"]), it
        assert np.array_equal(dist.view(np.uint64), g[f"dist{it}"].view(np.uint64)), it


@pytest.mark.parametrize("name", LLOYD)
def test_silhouette(name):
    # silhouette_cluster (silhouette.hpp:31-144) of every golden assignment, NaN bits included
    m, g = META[name], golden(name)
    X = case_rows(name)
    for it in range(len(g["cont"])):
        out, _ = oracle.silhouette(X, g[f"assign{it}"], g[f"centers{it}"], m["metric"])
        assert np.array_equal(out.view(np.uint64), g[f"sil{it}"].view(np.uint64)), it


@pytest.mark.parametrize("name", RANGE)
def test_range_silhouette(name):
    # silhouette_cluster of each range assignment (the reference's harness runs
    # it on the clusters lsh_/cube_range_assignment produced), NaN bits included
    m, g = META[name], golden(name)
    X = case_rows(name)
    for it in range(int(g["iters"][0])):
        out, _ = oracle.silhouette(X, g[f"assign{it}"], g[f"centers{it}"], m["metric"])
        assert np.array_equal(out.view(np.uint64), g[f"sil{it}"].view(np.uint64)), it


@pytest.mark.parametrize("name", cases("chain"))
def test_recommender_chain(name):
    # main.cpp:149-222: cosine LSH over user vectors (general doubles), filtered
    # combined buckets per user, get_P_closest, get_top_N_recom
    m, g = META[name], golden(name)
    pool = g["pool"]
    users = pool if m["self"] else g["users"]
    R, _ = oracle.gen_lsh_cosine(m["seed"], m["L"], m["k"], m["d"])
    assert np.array_equal(R.view(np.uint64), g["R"].view(np.uint64))
    b = oracle.lsh_hash_cosine(pool, R)
    assert np.array_equal(b, g["g"])
    nb = 1 << m["k"]
    rp, idx = oracle.bucket_csr(b, nb)
    qb = oracle.lsh_hash_cosine(users, R)
    lists = [oracle.lsh_query(m["N"], nb, rp, idx, qb[q]) for q in range(m["Q"])]
    ptr = np.cumsum([0] + [len(l) for l in lists]).astype(np.int64)
    cand = np.concatenate(lists).astype(np.int32)
    assert np.array_equal(ptr, g["nb_ptr"]) and np.array_equal(cand, g["nb_idx"])
    idx_, sim, cnt = oracle.p_closest(pool, users, ptr, cand, m["P"])
    assert np.array_equal(cnt, g["pc_cnt"]) and np.array_equal(idx_, g["pc_idx"])
    assert np.array_equal(sim.view(np.uint64), g["pc_sim"].view(np.uint64))
    up, ui = (g["punk_ptr"], g["punk_idx"]) if m["self"] else (g["uunk_ptr"], g["uunk_idx"])
    um = g["pmean"] if m["self"] else g["umean"]
    top = oracle.top_n_recom(pool, g["pmean"], users, um, up, ui, idx_, sim, cnt, m["NTOP"])
    has = cnt > 0
    assert np.array_equal(top[has], g["top"][has])


def crec_flow(X, K, iters, min_dist, rows, src_override=True):
    """main.cpp:248-254 / :340-347: Lloyd + k_means from dataset-row centroids
    until k_means reports no move or `iters`; returns (assign, centers, iterations)."""
    C = X[rows].astype(np.float64)
    it, cont, a = 0, True, None
    while cont and it < iters:
        a, _ = oracle.lloyd_assign(X, C, "euclidean", rows.astype(np.int32) if (it == 0 and src_override) else None)
        Cn, _, cont = oracle.kmeans_update(X, a, C, "euclidean", min_dist)
        C = Cn if cont else C
        it += 1
    return a, C, it


@pytest.mark.parametrize("name", cases("crec"))
def test_clustering_recommenders(name):
    # main.cpp's clustering recommenders on user-vector doubles, both parts, with
    # the 3-argument get_top_N_recom (crypto_rec.hpp:327-345) over whole clusters
    m, g = META[name], golden(name)
    K = m["K"]
    users, fake = g["users"], g["fake"]
    # Part A (main.cpp:240-273): rand_selection, Lloyd/k_means, each user's own cluster
    rows = oracle.rand_selection(m["N"], K, m["seedA"])
    assert np.array_equal(rows, g["A_rows"])
    a, C, it = crec_flow(users, K, m["iters"], m["min_dist"], rows)
    assert it == int(g["A_iters"][0]) and np.array_equal(a, g["A_assign"])
    assert np.array_equal(C.view(np.uint64), g["A_centers"].view(np.uint64))
    crow, crows = oracle.clusters_csr(a, K)
    top = oracle.cluster_top_n(users, g["umean"], crow, crows, users, g["umean"], a, g["uunk_ptr"], g["uunk_idx"],
                               m["NTA"])
    assert np.array_equal(top, g["A_top"])
    # Part B (main.cpp:334-381): k_means_pp over the fake users, the nearest
    # centroid of each user (the inline argmin :356-364 is lloyds_assignment's rule
    # without the override), recommendations from that cluster; empty ones skipped
    rows = oracle.kmeans_pp(fake, K, "euclidean", m["seedB"])
    assert np.array_equal(rows, g["B_rows"])
    a, C, it = crec_flow(fake, K, m["iters"], m["min_dist"], rows)
    assert it == int(g["B_iters"][0]) and np.array_equal(a, g["B_assign"])
    assert np.array_equal(C.view(np.uint64), g["B_centers"].view(np.uint64))
    ucl, _ = oracle.lloyd_assign(users, C, "euclidean", None)
    assert np.array_equal(ucl, g["B_ucl"])
    crow, crows = oracle.clusters_csr(a, K)
    top = oracle.cluster_top_n(fake, g["fmean"], crow, crows, users, g["umean"], ucl, g["uunk_ptr"], g["uunk_idx"],
                               m["NTB"])
    assert np.array_equal(top, g["B_top"])
