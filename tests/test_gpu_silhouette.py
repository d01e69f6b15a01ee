"""GPU parity: silhouette_cluster (silhouette.hpp:31-144) — per-cluster and
overall silhouettes bit-exact (NaN bits included: empty clusters, zero rows
under cosine) against the reference's golden outputs and the CPU oracle."""
import numpy as np
import pytest

import oracle
from amd import lshkm
from conftest import case_rows, cases, golden, golden_meta, lloyd_input

META = golden_meta()
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return lshkm.Context(0)


def to_dev(ctx, a):
    return ctx.torch.from_numpy(np.ascontiguousarray(a)).to(ctx.dev)


def bits(a):
    return np.asarray(a, np.float64).view(np.uint64)


@pytest.mark.parametrize("name", cases("lloyd"))
def test_silhouette_golden(ctx, name):
    m, g = META[name], golden(name)
    X = to_dev(ctx, lloyd_input(name))
    for it in range(len(g["cont"])):
        out, _ = lshkm.silhouette(ctx, X, to_dev(ctx, g[f"assign{it}"]), to_dev(ctx, g[f"centers{it}"]), m["metric"])
        assert np.array_equal(bits(out), bits(g[f"sil{it}"])), (it, out, g[f"sil{it}"])


@pytest.mark.parametrize("name", cases("range"))
def test_silhouette_range_golden(ctx, name):
    # the silhouettes of the reference's range assignments (lsh_/cube_range_assignment
    # clusters, incl. "k_means_center" centroids after an update)
    m, g = META[name], golden(name)
    X = to_dev(ctx, np.ascontiguousarray(case_rows(name)))
    for it in range(int(g["iters"][0])):
        out, _ = lshkm.silhouette(ctx, X, to_dev(ctx, g[f"assign{it}"]), to_dev(ctx, g[f"centers{it}"]), m["metric"])
        assert np.array_equal(bits(out), bits(g[f"sil{it}"])), (it, out, g[f"sil{it}"])


@pytest.mark.parametrize("N,d,K,metric,zero_every,kind", [
    (20_000, 128, 16, "euclidean", 0, "grid"),     # every square exact: the x*x form (grid test)
    (30_000, 16, 64, "euclidean", 0, "grid"),
    (12_000, 64, 12, "cosine", 101, "grid"),       # zero rows: NaN distances
    (5_000, 8, 300, "euclidean", 0, "grid"),       # many small (and some empty) clusters
    (12_000, 128, 10, "euclidean", 0, "normal"),   # full mantissas: glibc's pow where x*x may differ
    (6_000, 40, 24, "euclidean", 0, "wide"),       # a grid wider than 26 bits (x*x exact for most, not all)
])
def test_silhouette_vs_oracle(ctx, N, d, K, metric, zero_every, kind):
    Xh = oracle.synth(900 + d, N, d, kind="normal" if kind == "normal" else "grid")
    if kind == "wide":
        Xh[::7, 3] *= np.float32(2.0 ** 12)                 # spans 2^-15 .. 2^15: differences of up to 31 bits
    if zero_every:
        Xh[3::zero_every] = 0.0
    src = (np.arange(K) * (N // K)).astype(np.int32)
    C = Xh[src].astype(np.float64)
    X = to_dev(ctx, Xh)
    a, _ = lshkm.lloyd_assign(ctx, X, to_dev(ctx, C), metric, src)
    ah = a.cpu().numpy()
    out, s = lshkm.silhouette(ctx, X, a, to_dev(ctx, C), metric)
    oout, os_ = oracle.silhouette(Xh, ah, C, metric)
    assert np.array_equal(bits(s.cpu().numpy()), bits(os_))
    assert np.array_equal(bits(out), bits(oout))
