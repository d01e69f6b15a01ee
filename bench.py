"""Headline benchmark: point hash+assign ops/sec at d=128, N=10M per GPU, K=256.

--workload c3 (default; BASELINE.json configs[2] + the C2 hashing): one step =
  one pass of the hot path over the rank's resident shard: LSH hashing (L=5
  tables x k=4 EuclideanH functions, w=0.4, nb = N_total/100: k-tuples + bucket
  IDs) + Lloyd assignment over K=256 centroids (cluster ID + exact-order fp64
  distance). Multi-GPU: contiguous row shards, one process per GPU, no
  data-path collective (hash and assign are per point) -> weak scaling.
--workload c5 (configs[4]: 80M x 128, K=1024 over 8 GPUs = 10M per GPU): one
  step = one full iteration, sharding.ShardedLloyd: lshkm_hash_assign (K=1024)
  + lshkm_kmeans_partial + all-reduce of the K x d sums and K counts over RCCL
  + lshkm_kmeans_finalize (centers replaced as k_means does).
Points are synthetic (include/lshkm_synth.h), generated in HBM before timing.

python bench.py --gpus N --steps K --warmup W [--workload c5]   (torch.distributed.run for N>1)
"""
import argparse
import ctypes as C
import importlib.util
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
D, L_TABLES, K_FUNCS, W, BUCKET_DIV, SEED_DATA, SEED_PARAMS = 128, 5, 4, 0.4, 100, 0x5EED, 12345
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
F16_MFMA_PEAK_TFS = 2500.0     # MI355X_MICROARCH.md: FP16/BF16 MFMA dense peak


def load_module(name, fname):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "crypto-recommendation_amd", fname))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def load_pkg():
    return load_module("lshkm_amd", "lshkm.py")


sharding = load_module("lshkm_sharding", "sharding.py")


def port_all_cores(sample_hash, sample_assign, K):
    """The C restatement (oracle/_ref/liboracle.so, -O2, OpenMP over rows) on all
    of this rank's host cores (OMP_NUM_THREADS, 16 on the GPU box), in a child
    process so the thread count is set before the library loads."""
    cores = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    env = dict(os.environ, OMP_NUM_THREADS=str(cores))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "bench_port.py"), str(sample_hash),
                          str(sample_assign), str(K), str(SEED_DATA)], check=True, capture_output=True, text=True,
                         env=env).stdout
    res = json.loads(out.strip().splitlines()[-1])
    per_pt = res["hash_s"] / res["hash_pts"] + res["assign_s"] / res["assign_pts"]
    return {"value": 1.0 / per_pt, "unit": "point hash+assign ops/s", "cores": cores, "kind": "port",
            "sample": f"{res['hash_pts']} pts hashed (L=5,k=4) + {res['assign_pts']} pts assigned (K={K}), d=128, "
                      f"{cores} OpenMP threads, C restatement at -O2; hash {res['hash_s']:.2f}s, "
                      f"assign {res['assign_s']:.2f}s"}


def cpu_baseline(sample_hash, sample_assign, K):
    """The reference's own CPU path (oracle/_ref/ref_harness: g++ -O0 as shipped,
    1 thread) on a bounded sample; falls back to the C restatement (port)."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if os.path.exists(harness):
        out = subprocess.run([harness, "bench", str(sample_hash), str(sample_assign), str(K), str(SEED_DATA)],
                             check=True, capture_output=True, text=True).stdout
        res = json.loads(out.strip().splitlines()[-1])
        kind, cores = "reference", 1
    else:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        os.environ.setdefault("OMP_NUM_THREADS", "1")
        X = oracle.synth(SEED_DATA, max(sample_hash, sample_assign), D)
        V, t, r, _ = oracle.gen_lsh_euclid(SEED_PARAMS, L_TABLES, K_FUNCS, D, np.float32(W))
        t0 = time.perf_counter()
        oracle.lsh_hash_euclid(X[:sample_hash], V, t, np.float32(W), r, max(sample_hash // BUCKET_DIV, 1))
        t1 = time.perf_counter()
        rows = np.arange(K) * (sample_assign // K)
        oracle.lloyd_assign(X[:sample_assign], X[rows].astype(np.float64), "euclidean", rows.astype(np.int32))
        t2 = time.perf_counter()
        res = dict(hash_pts=sample_hash, hash_s=t1 - t0, assign_pts=sample_assign, assign_s=t2 - t1)
        kind, cores = "port", int(os.environ.get("OMP_NUM_THREADS", "1"))
    per_pt = res["hash_s"] / res["hash_pts"] + res["assign_s"] / res["assign_pts"]
    return {
        "value": 1.0 / per_pt, "unit": "point hash+assign ops/s", "cores": cores, "kind": kind,
        "sample": f"{res['hash_pts']} pts hashed (L=5,k=4) + {res['assign_pts']} pts assigned (K={K}), d=128, "
                  f"1 thread, {platform.processor() or platform.machine()}; hash {res['hash_s']:.2f}s, "
                  f"assign {res['assign_s']:.2f}s",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=10_000_000, help="points per GPU")
    ap.add_argument("--workload", choices=["c3", "c5"], default="c3")
    ap.add_argument("--k", type=int, default=None, help="centroids (default 256 for c3, 1024 for c5)")
    ap.add_argument("--cpu-port-hash-sample", type=int, default=400_000)
    ap.add_argument("--cpu-port-assign-sample", type=int, default=300_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-hash-sample", type=int, default=100_000)
    ap.add_argument("--cpu-assign-sample", type=int, default=12_000)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-launch HBM bytes measured by rocprofv3 PMC passes (see profiles/)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    lk = load_pkg()
    ctx = lk.Context(local)
    lib = lk.lib()
    N = args.n
    K = args.k or (1024 if args.workload == "c5" else 256)
    N_total = N * world
    nb = N_total // BUCKET_DIV

    # Resident shard + parameters (untimed).
    X = ctx.synth(SEED_DATA, N, D, row0=rank * N)
    V, t, r, _ = lk.params_lsh_euclidean(SEED_PARAMS, L_TABLES, K_FUNCS, D, W)
    lsh = lk.LSH(ctx, "euclidean", D, K_FUNCS, L_TABLES, nb, W, V=V, t=t, r=r)
    rows = sharding.centroid_rows(N_total, K)                      # reference init: rows i*floor(N/K)
    Cc = torch.empty((K, D), dtype=torch.float64, device=dev)
    for i, row in enumerate(rows):                                 # centroids may live on other shards
        Cc[i] = ctx.synth(SEED_DATA, 1, D, row0=int(row))[0].double()
    src = sharding.local_src_rows(rows, rank * N, N)               # centroid override, shard-local
    tuples = torch.empty((N, L_TABLES, K_FUNCS), dtype=torch.int32, device=dev)
    bucket = torch.empty((N, L_TABLES), dtype=torch.int32, device=dev)
    assign = torch.empty((N,), dtype=torch.int32, device=dev)
    dist_ = torch.empty((N,), dtype=torch.float64, device=dev)
    p = lambda t_: C.c_void_p(t_.data_ptr())
    src_p = src.ctypes.data_as(C.c_void_p)

    if args.workload == "c5":
        # one full iteration: hash + assign, per-shard sums, RCCL all-reduce, finalize
        del tuples, bucket, assign, dist_
        it = sharding.ShardedLloyd(lk, ctx, lsh, X, Cc, src, mode="fast")

        def step():
            it.step()
    else:
        def step():
            # one pass: tuples + bucket IDs + cluster IDs + fp64 distances (lshkm_hash_assign)
            lk._ck(lib.lshkm_hash_assign(lsh.h, p(X), N, p(Cc), K, src_p, p(tuples), None, p(bucket), p(assign),
                                         p(dist_)))

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        step()
    barrier()
    ctx.reset_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(e, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(e.item())
    ambig = ctx.stat(lk.STAT_ASSIGN_AMBIG) // args.steps
    hexact = ctx.stat(lk.STAT_HASH_EXACT) // args.steps
    hfix = ctx.stat(lk.STAT_HASH_FIX) // args.steps

    # Dominant kernel = the fused pass (fused_persistent_kernel<true> and its
    # hash_fixup_kernel; at K > 256 one launch per 256-centroid slice): HIP
    # events recorded by the library around those launches, on the stream they
    # run on; averaged over reps steps.
    reps = max(3, args.steps)
    lk._ck(lib.lshkm_ctx_enable_timing(ctx.h, 1))
    ms = C.c_float()
    t_kernel = 0.0
    for _ in range(reps):
        step()
        lk._ck(lib.lshkm_last_kernel_ms(ctx.h, C.byref(ms)))
        t_kernel += ms.value / 1e3
    lk._ck(lib.lshkm_ctx_enable_timing(ctx.h, 0))
    t_kernel /= reps

    # Algorithmic bytes and flops per point: 512 B read, 80 B tuples +
    # 20 B bucket IDs + 4 B cluster ID + 8 B distance written = 624 B; 2*d*(L*k + K) flop.
    bytes_per_pt = 4 * D + 4 * L_TABLES * K_FUNCS + 4 * L_TABLES + 4 + 8
    flop_per_pt = 2 * D * (L_TABLES * K_FUNCS + K)
    kpad = (K + 63) // 64 * 64
    # hi-only form: the hash tile's 3 split-f16 products (32 padded rows) + one
    # f16 product per centroid (padded tiles); the ~3% of rows the hi-only bound
    # leaves to the 3-product refinement are not counted
    mfma_flop_per_pt = 2 * D * (3 * 32 + kpad)
    hbm_gbs = bytes_per_pt * N / t_kernel / 1e9
    mfma_tfs = mfma_flop_per_pt * N / t_kernel / 1e12
    traffic = None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if tj.get("N") == N and tj.get("K") == K and tj.get("workload", "c3") == args.workload:
            traffic = tj.get("hbm_bytes_per_launch")

    if rank == 0:
        value = N_total * args.steps / elapsed
        line = {
            "metric": "point hash+assign ops/sec at d=128, N=10M, K=256; 1/2/4/8 MI355X",
            "value": value,
            "unit": "point hash+assign ops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32 points; split-f16 MFMA scores (f32 accumulate), fp64/x87-exact results",
            "data": "synthetic (include/lshkm_synth.h), resident in HBM",
            "config": {"workload": (f"C5 LSH-assign + k-means iteration (hash + assign + per-shard sums + RCCL "
                                    f"all-reduce + finalize), K={K}, N={N} per GPU, d=128"
                                    if args.workload == "c5" else
                                    f"C3 Lloyd K={K} + C2 LSH L=5 k=4 hashing, N={N} per GPU, d=128"),
                       "N_per_gpu": N, "N_total": N_total, "d": D, "K": K, "L": L_TABLES, "k": K_FUNCS,
                       "w": W, "nb": nb, "parallelism": f"dp{world} (row shards)"},
            "roofline": {
                "bound": "hbm",
                "kernel": "fused pass = fused_hi_kernel (hash + hi-only f16 centroid scores, one read of X) + "
                          "hash_fixup_kernel + the 3-product refinement of the rows the hi-only bound leaves",
                "achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "bytes_per_point": bytes_per_pt, "kernel_ms": t_kernel * 1e3,
                "mfma": {"achieved_TFs": mfma_tfs, "peak_TFs": F16_MFMA_PEAK_TFS, "frac": mfma_tfs / F16_MFMA_PEAK_TFS,
                         "flop_per_point_executed": mfma_flop_per_pt, "flop_per_point_algorithmic": flop_per_pt},
            },
            "exactness": {"per_step": True, "assign_ambiguous_rows": ambig, "hash_fixup_rows": hfix,
                          "hash_exact_fallbacks": hexact},
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_hash_sample, args.cpu_assign_sample, K)
            try:
                line["cpu_baseline"]["all_cores"] = port_all_cores(args.cpu_port_hash_sample,
                                                                   args.cpu_port_assign_sample * 256 // K, K)
            except (subprocess.CalledProcessError, OSError, ValueError) as e:
                line["cpu_baseline"]["all_cores"] = {"error": str(e)[:200]}
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
