"""Cosine Lloyd timed per call (profiling aid): fp64 user-vector rows (1M x 100,
K = 256), or with --c3 the C3 shape (10M x 128 fp32 synthetic, K = 256)."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from amd import lshkm
ctx = lshkm.Context(0)
if "--c3" in sys.argv:
    N, d, K = 10_000_000, 128, 256
    X = ctx.synth(0x5EED + 4, N, d)
    C = X[torch.from_numpy((np.arange(K) * (N // K)).astype(np.int64)).to(ctx.dev)].double()
    metrics = ("cosine",)
else:
    rng = np.random.default_rng(11)
    N, d, K = 1_000_000, 100, 256
    X = torch.from_numpy(rng.standard_normal((N, d))).to(ctx.dev)
    C = X[torch.from_numpy((np.arange(K) * (N // K)).astype(np.int64)).to(ctx.dev)].clone()
    metrics = ("cosine", "euclidean")
for metric in metrics:
    lshkm.lloyd_assign(ctx, X, C, metric)
    ctx.sync()
    ctx.reset_stats()
    t0 = time.perf_counter()
    for _ in range(5):
        lshkm.lloyd_assign(ctx, X, C, metric)
    ctx.sync()
    print(metric, (time.perf_counter() - t0) / 5 * 1e3, "ms", "ambig", ctx.stat(lshkm.STAT_ASSIGN_AMBIG) / 5,
          "cosfix", ctx.stat(lshkm.STAT_COS_FIX) / 5, "refined", ctx.stat(lshkm.STAT_REFINED) / 5)
