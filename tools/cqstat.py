import sys, os, numpy as np, torch
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
from amd import lshkm
ctx = lshkm.Context(0)
N, d, k = 10_000_000, 128, 14
X = ctx.synth(0x5EED, N, d)
V, tt, st = lshkm.params_cube_euclidean(4242, k, d, 2.0)
cube = lshkm.Cube(ctx, "euclidean", d, k, 2.0, V=V, t=tt, rng_state=st)
cube.build(X)
nq = 65_536
Q = X[torch.arange(nq, device=ctx.dev) * (N // nq)]
ptr, out = cube.query(Q, 14, device=True)
rp, _ = cube.buckets()
sz = np.diff(rp)
print("total", int(ptr[-1].item()), "bucket max", sz.max(), "mean", sz.mean(), "nonempty", (sz > 0).sum(), "sum s^2/N", (sz.astype(np.float64) ** 2).sum() / N)
