# C5: per-iteration sizes of the recommend users' clusters and the
# (similarity, chain) phase times -- the first iteration's long chain.
import os, sys, time, importlib.util
import numpy as np, torch
ROOT = os.environ.get('GRAFT_REPO_ROOT', '/root/repo')
def load(name, f):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, 'crypto-recommendation_amd', f))
    m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m); return m
lk = load('lshkm_amd', 'lshkm.py'); sh = load('lshkm_sharding', 'sharding.py')
ctx = lk.Context(0); dev = torch.device('cuda', 0)
N, D, K = 10_000_000, 128, 1024
X = ctx.synth(0x5EED, N, D)
V, t, r, _ = lk.params_lsh_euclidean(12345, 5, 4, D, 0.4)
lsh = lk.LSH(ctx, 'euclidean', D, 4, 5, N // 100, 0.4, V=V, t=t, r=r)
rows = sh.centroid_rows(N, K)
Cc = torch.empty((K, D), dtype=torch.float64, device=dev)
for i, row in enumerate(rows): Cc[i] = ctx.synth(0x5EED, 1, D, row0=int(row))[0].double()
it = sh.ShardedLloyd(lk, ctx, lsh, X, Cc, sh.local_src_rows(rows, 0, N), mode='certified')
it.enable_recommend(N, 0, Q=1024, n_top=5)
it.recom_timing = []
for s in range(5):
    it.step(); torch.cuda.synchronize()
    ucl = it.recom_ucl.cpu().numpy(); cnt = it.last_counts.cpu().numpy()
    print('step', s, 'sims/chain ms', [round(x, 3) for x in it.recom_timing[-1]], 'user cluster sizes: max', cnt[ucl].max(),
          'mean', round(cnt[ucl].mean()), 'all clusters max', cnt.max(), 'sum', cnt[ucl].sum(), flush=True)
# step 0 again, every kernel already loaded (the first call's numbers include
# the code objects' first launches and the workspace allocations)
it = sh.ShardedLloyd(lk, ctx, lsh, X, Cc, sh.local_src_rows(rows, 0, N), mode='certified')
it.enable_recommend(N, 0, Q=1024, n_top=5)
it.recom_timing = []
it.step(); torch.cuda.synchronize()
print('step 0 (warm) sims/chain ms', [round(x, 3) for x in it.recom_timing[-1]], flush=True)
