"""The clustering recommender's terms phase at the C5 shape (10M fp32 rows,
d = 128, K = 1024 clusters, 1024 users; profiling aid): time per call, the
x87-decided similarity count."""
import os, sys, time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from amd import lshkm
ctx = lshkm.Context(0)
N, d, K, Q = int(os.environ.get("TT_N", 10_000_000)), 128, 1024, 1024
X = ctx.synth(0x5EED, N, d)
g = torch.Generator(device="cpu").manual_seed(3)
assign = torch.randint(0, K, (N,), generator=g, dtype=torch.int32).to(ctx.dev)
crow, crows = lshkm.clusters(ctx, assign, K)
rows = torch.arange(Q, dtype=torch.int64) * (N // Q)
U = X[rows.to(ctx.dev)].clone()
ucl = assign[rows.to(ctx.dev)].clone()
m = 8
up = torch.arange(Q + 1, dtype=torch.int64) * m
ui = torch.tensor([(16 * k + (q % 16)) % d for q in range(Q) for k in range(m)], dtype=torch.int32)
xm = torch.zeros(N, dtype=torch.float64, device=ctx.dev)
up, ui = up.to(ctx.dev), ui.to(ctx.dev)
for it in range(2):
    out = lshkm.cluster_terms(ctx, X, xm, crow, crows, U, ucl, up, ui)
ctx.sync()
ctx.reset_stats()
t0 = time.perf_counter()
for _ in range(3):
    out = lshkm.cluster_terms(ctx, X, xm, crow, crows, U, ucl, up, ui)
ctx.sync()
print(f"cluster_terms: {(time.perf_counter() - t0) / 3 * 1e3:.3f} ms per call; members {int(out[0][-1].item())}; "
      f"x87-decided {ctx.stat(7) // 3}", flush=True)
