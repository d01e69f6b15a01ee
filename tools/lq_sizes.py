"""Bucket-size distribution of the C2 index and the query pairs' candidate
counts (diagnostic for get_LSH_filtered_combined_buckets' load balance)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from amd import lshkm  # noqa: E402

ctx = lshkm.Context(0)
N, d, L, k = 1_000_000, 128, 5, 4
X = ctx.synth(0x5EED, N, d)
V, tt, r, _ = lshkm.params_lsh_euclidean(12345, L, k, d, 0.4)
lsh = lshkm.LSH(ctx, "euclidean", d, k, L, N // 100, 0.4, V=V, t=tt, r=r)
lsh.build(X)
bu = lsh.hash(X, tuples=False, phi=False)[2].cpu().numpy()
for l in range(L):
    c = np.bincount(bu[:, l], minlength=N // 100)
    print(f"table {l}: bucket size max {c.max()}, mean {c.mean():.1f}, sum n^2/N {float((c.astype(np.float64) ** 2).sum() / N):.1f}")
nq = 65_536
Q = X[torch.arange(nq, device=ctx.dev) * (N // nq)]
ptr, _ = lsh.query(Q, filtered=False)
sz = np.diff(ptr)
print("unfiltered candidates per query: total", int(ptr[-1]), "mean", sz.mean(), "max", sz.max(),
      "p99", np.percentile(sz, 99), "p50", np.median(sz), flush=True)
