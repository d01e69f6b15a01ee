import sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
from amd import lshkm
ctx = lshkm.Context(0)
X = ctx.synth(0x5EED, 1_000_000, 128)
ctx.reset_stats()
rows = lshkm.kmeans_pp_rows(ctx, X, 64, "euclidean", 7)
print("chunks", ctx.stat(2), "seq", ctx.stat(3), "per centroid", ctx.stat(3) / 63)
