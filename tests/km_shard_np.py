"""A numpy restatement of lshkm.ShardSums (the per-rank calls of the sharded
k-means sums, include/lshkm.h lshkm_kmeans_shard_*), so that the protocol in
sharding.kmeans_sums_sharded -- its collectives, rank order and carry -- runs
on CPU ranks over gloo (tests/test_sharding_gloo.py). Test infrastructure: the
GPU library's own calls are checked by tests/test_gpu_multirank.py.

The arithmetic follows csrc/update.hip: begin = any-order partial sums, sums
of |x|, the values' lowest set-bit exponent q and top bit position t;
certify = km_cert on the global values (the count form, then the |x| form);
chain = the reference's sequential fp64 chain (update.hpp:52-56) from the
carry over this rank's members of each flagged (c, j), in row order."""
import numpy as np
import torch

KMF_BAD = 1 << 20


def bit_positions(x):
    """(q, t) per element: the lowest set-bit exponent and the top bit position
    (+1) of each nonzero finite value (x = M 2^(e - 53), M a 53-bit integer)."""
    x = np.asarray(x, np.float64)
    m, e = np.frexp(np.abs(x))
    M = (m * 2.0 ** 53).astype(np.uint64)
    low = M & (~M + np.uint64(1))
    ctz = np.zeros(M.shape, np.int64)
    nz = M != 0
    ctz[nz] = np.log2(low[nz].astype(np.float64)).astype(np.int64)
    return e.astype(np.int64) - 53 + ctz, e.astype(np.int64)


def km_cert(q, t, cnt, asum):
    """csrc/update.hip km_cert, elementwise (q, t, asum [K][d]; cnt [K])."""
    q, t = np.asarray(q, np.int64), np.asarray(t, np.int64)
    cnt = np.asarray(cnt, np.int64)[:, None] * np.ones_like(q)
    lc = np.ceil(np.log2(np.maximum(cnt, 1))).astype(np.int64)
    bad = q <= -KMF_BAD // 2
    empty = q > t
    count_form = (lc + t - q <= 53) & (lc + t <= 1023)
    with np.errstate(over="ignore"):
        lim = np.ldexp(1.0, np.minimum(53 + q, 1024).astype(np.int32))
        abs_form = asum * (1.0 + 2.0 ** -20) < lim
    return ~bad & (empty | count_form | abs_form)


class NumpyShardSums:
    """ShardSums' methods over one rank's rows X [n][d] and assignment a [n]."""

    def __init__(self, X, a, K):
        self.X, self.a, self.K = np.asarray(X), np.asarray(a), K
        self.d = self.X.shape[1]

    def empty(self, shape, dtype):
        return torch.empty(shape, dtype=dtype)

    def begin(self):
        K, d = self.K, self.d
        X64 = self.X.astype(np.float64)
        sums = np.zeros((K, d))
        asum = np.zeros((K, d))
        q = np.full((K, d), 1 << 30, np.int64)
        t = np.full((K, d), -(1 << 30), np.int64)
        counts = np.bincount(self.a, minlength=K).astype(np.int64)
        qv, tv = bit_positions(X64)
        finite = np.isfinite(X64)
        nz = (X64 != 0) & finite
        for c in range(K):
            rows = self.a == c
            if not rows.any():
                continue
            sums[c] = X64[rows][::-1].sum(axis=0)             # any order (here: reversed, pairwise)
            asum[c] = np.abs(X64[rows]).sum(axis=0)
            qq = np.where(nz[rows], qv[rows], 1 << 30).min(axis=0)
            q[c] = np.where((~finite[rows]).any(axis=0), -KMF_BAD, qq)
            t[c] = np.where(nz[rows], tv[rows], -(1 << 30)).max(axis=0)
        qt = np.stack([q, -t]).astype(np.int32)
        return (torch.from_numpy(sums), torch.from_numpy(asum), torch.from_numpy(qt), torch.from_numpy(counts))

    def certify(self, gathered, asum, qt, counts, world, rank):
        g = gathered.numpy()
        tot = np.zeros(g.shape[1:])
        pre = np.zeros(g.shape[1:])
        for r in range(world):                               # rank order
            if r == rank:
                pre = tot.copy()
            tot = tot + g[r]
        qt = qt.numpy().astype(np.int64)
        ok = km_cert(qt[0], -qt[1], counts.numpy(), asum.numpy())
        lane = ~ok & (counts.numpy()[:, None] <= 32768)           # one lane each (km_chain_lanes_kernel)
        mask = np.where(ok, 0, np.where(lane, 2, 1)).astype(np.uint8)
        flag = np.zeros(self.K, np.int32)
        for c, j in zip(*np.nonzero(mask == 1)):
            flag[c] |= np.int32(1 << min(31, j // 64))
        return (torch.from_numpy(tot), torch.from_numpy(pre), torch.from_numpy(flag), torch.from_numpy(mask),
                int((~ok).sum()))

    def prepare(self, start, flag, mask):
        pass                                                 # the segment records: a device-side speedup only

    def chain(self, flag, mask, carry, sums):
        X64 = self.X.astype(np.float64)
        m = mask.numpy().astype(bool)
        out = sums.numpy()
        for c, j in zip(*np.nonzero(m)):
            s = 0.0 if carry is None else float(carry.numpy()[c, j])
            vals = X64[self.a == c, j]
            if len(vals):
                s = np.cumsum(np.concatenate([[s], vals]))[-1]    # strictly in order
            out[c, j] = s
