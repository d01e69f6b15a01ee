"""Time k-means++ seeding (lshkm_kmeans_pp) at bench scale and report how the
exact prefix-sum walk resolved its chunks. Profiling aid.
Env: KP_N (10M), KP_D (128), KP_K (32), KP_METRIC (euclidean)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from amd import lshkm  # noqa: E402

N = int(os.environ.get("KP_N", 10_000_000))
D = int(os.environ.get("KP_D", 128))
K = int(os.environ.get("KP_K", 32))
METRIC = os.environ.get("KP_METRIC", "euclidean")
ctx = lshkm.Context(0)
X = ctx.synth(0x5EED, N, D)
torch.cuda.synchronize()
lshkm.kmeans_pp_rows(ctx, X, 2, METRIC, 7)          # warm-up (module load)
ctx.reset_stats()
t0 = time.perf_counter()
rows = lshkm.kmeans_pp_rows(ctx, X, K, METRIC, 7)
dt = time.perf_counter() - t0
chunks, seq = ctx.stat(2), ctx.stat(3)
print(f"kmeans_pp N={N} d={D} K={K} {METRIC}: {dt * 1e3:.1f} ms total, {dt * 1e3 / max(K - 1, 1):.3f} ms/centroid, "
      f"chunks {chunks}, element-wise {seq} ({seq / max(K - 1, 1):.1f}/centroid), rows[:8] {rows[:8].tolist()}",
      flush=True)
