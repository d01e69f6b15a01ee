"""Diagnostic: where does the fused hash disagree with the oracle? (GPU box)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402
from amd import lshkm  # noqa: E402

ctx = lshkm.Context(0)
for N in (int(a) for a in sys.argv[1:] or ["200003"]):
    d, L, k, K, w = 128, 5, 4, 256, 0.4
    V, t, r, _ = lshkm.params_lsh_euclidean(12345, L, k, d, w)
    X = ctx.synth(0x5EED, N, d)
    lsh = lshkm.LSH(ctx, "euclidean", d, k, L, N // 100, w, V=V, t=t, r=r)
    rows = (np.arange(K) * (N // K)).astype(np.int32)
    Cc = X[torch.from_numpy(rows.astype(np.int64)).to(X.device)].double()
    tu, ph, bu, a, dist = lshkm.hash_assign(lsh, X, Cc, rows, tuples=True, phi=True, bucket=True)
    torch.cuda.synchronize()
    Xh = X.cpu().numpy()
    xt, xp, xb = oracle.lsh_hash_euclid(Xh, V, t, np.float32(w), r, N // 100)
    g = tu.cpu().numpy().reshape(N, L * k)
    o = xt.reshape(N, L * k)
    bad = np.argwhere(g != o)
    print(f"N={N}: {len(bad)} mismatching hash values in {len(np.unique(bad[:, 0]))} rows")
    Vf = V.reshape(L * k, d).astype(np.float64)
    tf = t.reshape(L * k).astype(np.float64)
    for row, f in bad[:12]:
        y = (Vf[f] @ Xh[row].astype(np.float64) + tf[f]) / np.float64(np.float32(w))
        print(f"  row {row} (tile {row // 32}, lane {row % 32}) f {f}: gpu {g[row, f]} oracle {o[row, f]} y {y:.6f}")
    if len(bad):
        rr = np.unique(bad[:, 0])
        print("  rows mod 32 histogram:", np.bincount(rr % 32, minlength=32).tolist())
        print("  fns histogram:", np.bincount(bad[:, 1], minlength=L * k).tolist())
