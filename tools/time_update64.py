"""k-means update on fp64 user-vector rows (1M x 100, K = 256), timed per call (profiling aid)."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from amd import lshkm
ctx = lshkm.Context(0)
rng = np.random.default_rng(11)
N, d, K = 1_000_000, 100, 256
X = torch.from_numpy(rng.standard_normal((N, d))).to(ctx.dev)
C = X[torch.from_numpy((np.arange(K) * (N // K)).astype(np.int64)).to(ctx.dev)].clone()
asg, _ = lshkm.lloyd_assign(ctx, X, C, "euclidean")
lshkm.kmeans_update(ctx, X, asg, C, "euclidean", 0.05)
ctx.sync()
t0 = time.perf_counter()
for _ in range(5):
    lshkm.kmeans_update(ctx, X, asg, C, "euclidean", 0.05)
ctx.sync()
print("update fp64", (time.perf_counter() - t0) / 5 * 1e3, "ms")
cnt = np.bincount(asg.cpu().numpy(), minlength=K)
print("cluster sizes: max", int(cnt.max()), "mean", float(cnt.mean()))
