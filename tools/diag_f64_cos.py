"""Diagnostic: cosine Lloyd on general fp64 rows vs the oracle, fresh context;
prints the mismatching rows with the oracle's distances to both centroids."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np

import oracle
from amd import lshkm
from test_gpu_f64 import _general_rows

N, d, K = 200_000, 100, 64
Xh = _general_rows(12, N, d)
rows = (np.arange(K) * (N // K)).astype(np.int32)
Ch = Xh[rows]
sub = 40_000
oa, od = oracle.lloyd_assign(Xh[:sub], Ch, "cosine", rows)
for path in ("auto", "exact", "auto"):
    if path == "exact":
        os.environ["LSHKM_ASSIGN_PATH"] = "exact"
    else:
        os.environ.pop("LSHKM_ASSIGN_PATH", None)
    ctx = lshkm.Context(0)
    X = ctx.torch.from_numpy(Xh).to(ctx.dev)
    ctx.reset_stats()
    a, dist = lshkm.lloyd_assign(ctx, X[:sub], ctx.torch.from_numpy(Ch).to(ctx.dev), "cosine", rows)
    a = a.cpu().numpy(); dist = dist.cpu().numpy()
    bad = np.nonzero(a != oa)[0]
    print(path, "mismatches", len(bad), "ambig", ctx.stat(lshkm.STAT_ASSIGN_AMBIG), "cosfix", ctx.stat(lshkm.STAT_COS_FIX),
          flush=True)
    for r in bad[:10]:
        dg = oracle.lloyd_assign(Xh[r:r + 1], Ch[[a[r]]], "cosine")[1][0]
        do = oracle.lloyd_assign(Xh[r:r + 1], Ch[[oa[r]]], "cosine")[1][0]
        print(f"  row {r}: gpu {a[r]} (oracle dist {dg!r}, gpu dist {dist[r]!r}) oracle {oa[r]} ({do!r}) "
              f"|x|={np.linalg.norm(Xh[r]):.3e}", flush=True)
    del X
    ctx.close()
    print("closed", flush=True)
print("done", flush=True)
