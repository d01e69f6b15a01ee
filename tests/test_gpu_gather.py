"""GPU: the winner-row sources of the K <= 256 distance chain agree bit for bit.

fused_hi_kernel<..., GATH> gathers the winners' centroid rows into LDS by
LDS-DMA: the f32 image when every centroid value is an f32 (dataset rows, the
first Lloyd iteration; exact as doubles), else the fp64 rows; the test build's
LSHKM_GATHER32=0 forces the fp64 rows, LSHKM_GATHER=0 register loads. All three
must give the reference-order distances (assignment.hpp:54-80,
cust_vector.hpp:124-136)."""
import numpy as np
import pytest

import oracle
from amd import lshkm
from conftest import assert_dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return lshkm.Context(0)


def run(M, ctx, monkeypatch, X, C, env, lsh_args=None):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if lsh_args is not None:
        lsh = M.LSH(ctx, "euclidean", *lsh_args[0], **lsh_args[1])
        tu, _, bu, a, d = M.hash_assign(lsh, X, C, tuples=True, bucket=True)
        out = (tu.cpu().numpy(), bu.cpu().numpy(), a.cpu().numpy(), d.cpu().numpy())
    else:
        a, d = M.lloyd_assign(ctx, X, C, "euclidean")
        out = (a.cpu().numpy(), d.cpu().numpy())
    for k in env:
        monkeypatch.delenv(k)
    return out


@pytest.mark.parametrize("K,general,hashing", [(256, False, True), (256, True, True), (200, False, False), (64, True, False)])
def test_gather_modes_agree(ctx, sctx, sw, monkeypatch, K, general, hashing):
    # the gather feeds the exact winner chain: the LSHKM_DIST_EXACT contract
    ctx.set_dist_mode("exact")
    sctx.set_dist_mode("exact")
    N, d = 300_007, 128
    X = ctx.synth(0x6A7 + K, N, d)
    Xh = X.cpu().numpy()
    rng = np.random.default_rng(K)
    Ch = Xh[rng.choice(N, K, replace=False)].astype(np.float64)
    Ch[9] = Ch[4]
    if general:
        Ch[K - 1] *= 1.0 + 2.0 ** -40            # one value not an f32: the fp64 rows for all
    C = ctx.torch.from_numpy(Ch).to(ctx.dev)
    lsh_args = None
    if hashing:
        V, t, r, _ = lshkm.params_lsh_euclidean(77, 5, 4, d, 0.4)
        lsh_args = ((d, 4, 5, N // 100, 0.4), dict(V=V, t=t, r=r))
    ref = run(lshkm, ctx, monkeypatch, X, C, {}, lsh_args)
    for env in ({"LSHKM_GATHER32": "0"}, {"LSHKM_GATHER": "0"}):
        got = run(sw, sctx, monkeypatch, X, C, env, lsh_args)
        for g, w in zip(got, ref):
            assert np.array_equal(g.view(np.uint8), w.view(np.uint8)), env
    sub = np.random.default_rng(2).choice(N, 2000, replace=False)
    oa, od = oracle.lloyd_assign(Xh[sub], Ch, "euclidean", None)
    a, dist = ref[-2], ref[-1]
    assert np.array_equal(a[sub], oa)
    assert_dist(dist[sub], od, "exact")          # general centroids too: glibc's pow(x, 2)
    ctx.set_dist_mode("certified")
    sctx.set_dist_mode("certified")
