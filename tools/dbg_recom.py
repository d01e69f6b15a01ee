"""Debug aid: the recom_f64 golden case on the GPU, every similarity that
differs from the fixture dumped to gpurun_out/dbg_recom.npz (user, position,
GPU value, fixture value, and the raw similarity array of the candidate list)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from amd import lshkm  # noqa: E402
from conftest import golden, golden_meta  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "recom_f64"
m, g = golden_meta()[name], golden(name)
ctx = lshkm.Context(0)
t = ctx.torch


def dev(a):
    return t.from_numpy(np.ascontiguousarray(a)).to(ctx.dev)


idx, sim, cnt = lshkm.p_closest(ctx, dev(g["x"]), dev(g["u"]), dev(g["cand_ptr"]), dev(g["cand_idx"]), m["P"])
idx, sim, cnt = idx.cpu().numpy(), sim.cpu().numpy(), cnt.cpu().numpy()
bad = np.argwhere(sim.view(np.uint64) != g["pc_sim"].view(np.uint64))
print("differing entries:", len(bad))
for q, j in bad[:20]:
    print(q, j, idx[q, j], g["pc_idx"][q, j], repr(sim[q, j]), repr(g["pc_sim"][q, j]))
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/dbg_recom.npz", bad=bad, idx=idx, sim=sim, cnt=cnt)
