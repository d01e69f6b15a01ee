"""GPU parity on full-mantissa rows (fp32 N(0,1) data).

The grid generator (include/lshkm_synth.h, <= 18 significant bits) is the
best case for several certificates: the f16 hi/lo split of a row is exact,
every difference squares exactly, every k-means chain passes the never-rounds
test. The "normal" generator (Irwin-Hall(12), full 24-bit mantissas) is the
case the reference's real inputs are like: here the whole C3 / C5 pipeline --
hashing, bucket IDs, assignment (both distance modes) and several k-means
updates -- is checked against the oracle bit for bit. Reference:
lib/lsh_cube.hpp:44-74, lib/clustering_phases/assignment.hpp:54-80,
update.hpp:37-86.
"""
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


def test_normal_generator_matches_oracle(ctx):
    # three producers, one bit pattern: the device kernel, the C oracle, numpy
    X = ctx.synth(0x5EED, 3000, 128, row0=9_999_000, kind="normal").cpu().numpy()
    Xo = oracle.synth(0x5EED, 3000, 128, row0=9_999_000, kind="normal")
    Xn = oracle.synth_normal_np(0x5EED, 3000, 128, row0=9_999_000)
    assert np.array_equal(X.view(np.uint32), Xo.view(np.uint32))
    assert np.array_equal(X.view(np.uint32), Xn.view(np.uint32))
    assert abs(X.mean()) < 0.01 and abs(X.std() - 1.0) < 0.01
    lowbit = (X.view(np.uint32) & 0xFF) != 0                 # the low 8 mantissa bits in use
    assert lowbit.mean() > 0.95


@pytest.mark.parametrize("mode", ["certified", "exact"])
def test_c3_iterations_on_normal_rows(ctx, mode):
    # hash + assign (lshkm_hash_assign: tuples, buckets, IDs, distances) and the
    # k-means update over 3 iterations, the reference's init (rows i * N / K)
    N, d, L, k, K = 60_000, 128, 5, 4, 64
    X = ctx.synth(0x5EED, N, d, kind="normal")
    Xh = X.cpu().numpy()
    V, t, r, _ = lshkm.params_lsh_euclidean(12345, L, k, d, 0.4)
    lsh = lshkm.LSH(ctx, "euclidean", d, k, L, N // 100, 0.4, V=V, t=t, r=r)
    xt, _, xb = oracle.lsh_hash_euclid(Xh, V, t, np.float32(0.4), r, N // 100)
    rows = (np.arange(K) * (N // K)).astype(np.int32)
    C = X[ctx.torch.from_numpy(rows.astype(np.int64)).to(ctx.dev)].double()
    src = rows
    ctx.set_dist_mode(mode)
    ctx.reset_stats()
    try:
        for it in range(3):
            tu, _, bu, a, dist = lshkm.hash_assign(lsh, X, C, src)
            oa, od = oracle.lloyd_assign(Xh, C.cpu().numpy(), "euclidean", src)
            assert np.array_equal(tu.cpu().numpy(), xt) and np.array_equal(bu.cpu().numpy(), xb)
            assert np.array_equal(a.cpu().numpy(), oa), it
            assert_dist(dist.cpu().numpy(), od, mode)
            Cn, cnt, cont = lshkm.kmeans_update(ctx, X, a, C, "euclidean", 0.0)
            Co, co, conto = oracle.kmeans_update(Xh, oa, C.cpu().numpy(), "euclidean", 0.0)
            assert np.array_equal(Cn.cpu().numpy().view(np.uint64), Co.view(np.uint64)), it
            assert np.array_equal(cnt.cpu().numpy(), co) and bool(cont) == bool(conto)
            C, src = Cn, None
    finally:
        ctx.set_dist_mode("certified")
    # full mantissas reach the certificates: the fix-up paths ran
    assert ctx.stat(lshkm.STAT_HASH_FIX) > 0
