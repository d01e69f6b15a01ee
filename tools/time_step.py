"""Per-call host enqueue time vs GPU time of bench.py's C3 step (lshkm_hash_assign
with and without the centroid override), to see which bounds ms_per_step."""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from amd import lshkm  # noqa: E402

N, D, K, L, KF = 10_000_000, 128, 256, 5, 4
ctx = lshkm.Context(0)
lib = lshkm.lib()
X = ctx.synth(0x5EED, N, D)
V, t, r, _ = lshkm.params_lsh_euclidean(12345, L, KF, D, 0.4)
lsh = lshkm.LSH(ctx, "euclidean", D, KF, L, N // 100, 0.4, V=V, t=t, r=r)
rows = (np.arange(K) * (N // K)).astype(np.int32)
Cc = X[torch.from_numpy(rows.astype(np.int64)).to(X.device)].double()
dev = X.device
tuples = torch.empty((N, L, KF), dtype=torch.int32, device=dev)
bucket = torch.empty((N, L), dtype=torch.int32, device=dev)
assign = torch.empty((N,), dtype=torch.int32, device=dev)
dist = torch.empty((N,), dtype=torch.float64, device=dev)
p = lambda x: C.c_void_p(x.data_ptr())
for src in (rows, None):
    sp = src.ctypes.data_as(C.c_void_p) if src is not None else None
    call = lambda: lshkm._ck(lib.lshkm_hash_assign(lsh.h, p(X), N, p(Cc), K, sp, p(tuples), None, p(bucket),
                                                   p(assign), p(dist)))
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(20):
        h0 = time.perf_counter()
        call()
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 20
    print(f"src={'rows' if src is not None else 'none'}: wall {wall * 1e3:.3f} ms/call, host enqueue median "
          f"{np.median(host) * 1e3:.3f} ms, max {max(host) * 1e3:.3f} ms", flush=True)
