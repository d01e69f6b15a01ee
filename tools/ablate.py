"""Profiling aid: time the fused pass with parts of the persistent kernel switched
off (LSHKM_FUSED_ABLATE bits: 1 = re-read tile 0's rows (no HBM stream), 2 = no
hash tile, 4 = no centroid tiles, 8 = no distance chain). Results are NOT valid
under ablation; this only attributes time."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from amd import lshkm  # noqa: E402

N, D, K, L, KF = int(os.environ.get("ABL_N", 10_000_000)), 128, 256, 5, 4
ctx = lshkm.Context(0)
lib = lshkm.lib()
X = ctx.synth(0x5EED, N, D)
V, t, r, _ = lshkm.params_lsh_euclidean(12345, L, KF, D, 0.4)
lsh = lshkm.LSH(ctx, "euclidean", D, KF, L, N // 100, 0.4, V=V, t=t, r=r)
rows = (np.arange(K) * (N // K)).astype(np.int64)
Cc = X[torch.from_numpy(rows).to(X.device)].double()
dev = X.device
tuples = torch.empty((N, L, KF), dtype=torch.int32, device=dev)
bucket = torch.empty((N, L), dtype=torch.int32, device=dev)
assign = torch.empty((N,), dtype=torch.int32, device=dev)
dist = torch.empty((N,), dtype=torch.float64, device=dev)
p = lambda x: C.c_void_p(x.data_ptr())
lshkm._ck(lib.lshkm_ctx_enable_timing(ctx.h, 1))
ms = C.c_float()
for bits in [0, 1, 2, 4, 8, 2 | 8, 4 | 8, 2 | 4 | 8, 1 | 2 | 4 | 8, 1 | 2, 1 | 4, 1 | 8]:
    os.environ["LSHKM_FUSED_ABLATE"] = str(bits)
    ts = []
    for it in range(6):
        lshkm._ck(lib.lshkm_hash_assign(lsh.h, p(X), N, p(Cc), K, None, p(tuples), None, p(bucket), p(assign), p(dist)))
        lshkm._ck(lib.lshkm_last_kernel_ms(ctx.h, C.byref(ms)))
        if it >= 2:
            ts.append(ms.value)
    print(f"ablate={bits:2d}  fused pass {np.median(ts):.3f} ms", flush=True)
