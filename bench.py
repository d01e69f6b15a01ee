"""Headline benchmark: point hash+assign ops/sec at d=128, N=10M per GPU, K=256.

--workload c3 (default; BASELINE.json configs[2] + the C2 hashing): one step =
  one pass of the hot path over the rank's resident shard: LSH hashing (L=5
  tables x k=4 EuclideanH functions, w=0.4, nb = N_total/100: k-tuples + bucket
  IDs) + Lloyd assignment over K=256 centroids (cluster ID + exact-order fp64
  distance). Multi-GPU: contiguous row shards, one process per GPU, no
  data-path collective (hash and assign are per point) -> weak scaling.
  The same line carries a "c5" object (unless --no-c5): configs[4]'s full
  iteration on the same resident shard, below.
--workload c5 (configs[4]: 80M x 128, K=1024 over 8 GPUs = 10M per GPU): one
  step = one full iteration, sharding.ShardedLloyd: lshkm_hash_assign (K=1024)
  + lshkm_kmeans_partial + all-reduce of the K x d sums and K counts over RCCL
  + lshkm_kmeans_finalize (centers replaced as k_means does) + the recommend
  step ("k-means recommend"): --recom-users Q query users (rows spread over the
  whole job) get get_top_N_recom over their whole clusters (crypto_rec.hpp:
  327-345): similarities on every rank, prediction sums carried rank to rank
  over RCCL point-to-point (sharding.recommend_sharded).
Points are synthetic (include/lshkm_synth.h), generated in HBM before timing.

python bench.py --gpus N --steps K --warmup W [--workload c5]
  N > 1: started under torch.distributed.run (the driver does this), or, when
  no WORLD_SIZE is set, this script launches torch.distributed.run itself, as a
  child process, before anything touches the GPU. --dry-run: the same launch
  with the gloo backend and no GPU work (CPU test of the multi-rank plumbing).
"""
import argparse
import ctypes as C
import importlib.util
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
D, L_TABLES, K_FUNCS, W, BUCKET_DIV, SEED_DATA, SEED_PARAMS = 128, 5, 4, 0.4, 100, 0x5EED, 12345
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
F16_MFMA_PEAK_TFS = 2500.0     # MI355X_MICROARCH.md: FP16/BF16 MFMA dense peak
METRIC = "point hash+assign ops/sec at d=128, N=10M, K=256; 1/2/4/8 MI355X"
DTYPE = ("fp32 points; split-f16 MFMA scores (f32 accumulate); tuples, bucket IDs and cluster IDs bit-exact "
         "(x87-exact hashing, certified argmin); distances: certified f32, <= 2^-20 relative to the reference's "
         "fp64 (north star: 1e-5; the context's default LSHKM_DIST_CERTIFIED mode), LSHKM_DIST_EXACT for the "
         "reference-order fp64 chain (exactness.exact_distances)")
# algorithmic bytes per point of the fused pass: 512 B read, 80 B
# tuples + 20 B bucket IDs + 4 B cluster ID + 8 B distance written
BYTES_PER_PT = 4 * D + 4 * L_TABLES * K_FUNCS + 4 * L_TABLES + 4 + 8
DATA = {"grid": "synthetic (include/lshkm_synth.h grid generator: Irwin-Hall(4) on a 2^-15 grid), resident in HBM",
        "normal": "synthetic (include/lshkm_synth.h normal generator: Irwin-Hall(12), full fp32 mantissas), "
                  "resident in HBM"}


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


def attach_cpu_baseline(line, args, K):
    """line["cpu_baseline"] (+ line["c5"]["cpu_baseline"]): the reference's CPU
    path on a bounded sample, 1 thread, plus the C restatement on all cores."""
    line["cpu_baseline"] = cpu_baseline(args.cpu_hash_sample, args.cpu_assign_sample * 256 // K, K)
    try:
        line["cpu_baseline"]["all_cores"] = port_all_cores(args.cpu_port_hash_sample,
                                                           args.cpu_port_assign_sample * 256 // K, K)
    except (subprocess.CalledProcessError, OSError, ValueError) as e:
        line["cpu_baseline"]["all_cores"] = {"error": str(e)[:200]}
    if "c5" in line:
        cb = cpu_baseline(args.cpu_hash_sample, args.cpu_assign_sample // 4, 1024)
        cb["note"] = ("hash + assign only: the reference's k_means update adds ~4d flops per point, "
                      "not timed here")
        line["c5"]["cpu_baseline"] = cb


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """--gpus N > 1 without a torch.distributed environment: run N ranks of this
    script under torch.distributed.run as a child process (nothing here has
    touched the GPU) and return its exit code."""
    # the ranks' arguments travel in the environment: torch.distributed.run's own
    # parser would take some of ours (--n) for abbreviations of its options
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", LSHKM_BENCH_ARGV=json.dumps(sys.argv[1:]))
    return subprocess.call(cmd, env=env)


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def timed(step, steps, warmup, world, dev):
    """W untimed steps, then exactly K steps bracketed by barrier + synchronize;
    returns the max over ranks of the elapsed seconds."""
    def barrier():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
    for _ in range(warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    barrier()
    return max_over_ranks(time.perf_counter() - t0, world, dev)


def dry_run(args, world, rank):
    """gloo, CPU only: the rank layout, the C5 exchange (sharding.allreduce_partials
    on K x d fp64 sums + K counts) and the max-over-ranks timing."""
    import torch.distributed as dist
    if "MASTER_ADDR" not in os.environ:             # a single rank started directly
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("gloo")
    assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)
    dev = torch.device("cpu")
    K = args.k or 1024
    row0, n = sharding.shard_range(args.n * world, world, rank)
    sums = torch.full((K, D), float(rank + 1), dtype=torch.float64)
    counts = torch.full((K,), rank + 1, dtype=torch.int64)

    def step():
        sums.fill_(float(rank + 1))
        counts.fill_(rank + 1)
        sharding.allreduce_partials(sums, counts)
    elapsed = timed(step, args.steps, args.warmup, world, dev)
    tot = world * (world + 1) // 2
    ok = bool(torch.all(sums == float(tot)) and torch.all(counts == tot))
    gathered = [None] * world
    dist.all_gather_object(gathered, (rank, row0, n))
    dist.barrier()
    if rank == 0:
        line = {"dry_run": True, "metric": METRIC, "n_gpus": world, "world_size": world, "steps": args.steps,
                "ms_per_step": elapsed / args.steps * 1e3, "allreduce_ok": ok,
                "shards": [{"rank": r, "row0": a, "n": b} for r, a, b in gathered],
                "backend": dist.get_backend()}
        if not args.no_cpu_baseline:
            attach_cpu_baseline(line, args, args.k or 256)
        print(json.dumps(line), flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


def fused_kernel_ms(lk, lib, ctx, step, reps):
    """Mean time of the fused pass (the HIP events the library records around the
    fused-family launches, on the stream they run on) over reps steps."""
    lk._ck(lib.lshkm_ctx_enable_timing(ctx.h, 1))
    ms = C.c_float()
    tot = 0.0
    for _ in range(reps):
        step()
        lk._ck(lib.lshkm_last_kernel_ms(ctx.h, C.byref(ms)))
        tot += ms.value
    lk._ck(lib.lshkm_ctx_enable_timing(ctx.h, 0))
    return tot / reps


def traffic_for(path, N, K, workload):
    if os.path.exists(path):
        with open(path) as f:
            tj = json.load(f)
        if tj.get("N") == N and tj.get("K") == K and tj.get("workload", "c3") == workload:
            return tj.get("hbm_bytes_per_launch")
    return None


def roofline(N, K, kernel_ms, traffic, what):
    kpad = (K + 63) // 64 * 64
    # hi-only form: the hash tile's 3 split-f16 products (32 padded rows) + one
    # f16 product per centroid (padded tiles); the few rows the hi-only bound
    # leaves to the 3-product refinement are not counted
    mfma_flop_per_pt = 2 * D * (3 * 32 + kpad)
    flop_per_pt = 2 * D * (L_TABLES * K_FUNCS + K)
    t = kernel_ms / 1e3
    gbs = BYTES_PER_PT * N / t / 1e9
    tfs = mfma_flop_per_pt * N / t / 1e12
    return {"bound": "hbm", "kernel": what, "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gbs / HBM_PEAK_GBS, "traffic": traffic, "bytes_per_point": BYTES_PER_PT, "kernel_ms": kernel_ms,
            "mfma": {"achieved_TFs": tfs, "peak_TFs": F16_MFMA_PEAK_TFS, "frac": tfs / F16_MFMA_PEAK_TFS,
                     "flop_per_point_executed": mfma_flop_per_pt, "flop_per_point_algorithmic": flop_per_pt}}


FUSED_WHAT = ("fused pass = fused_centroid_prep + fused_hi_kernel (hash + hi-only f16 centroid scores, one read of X "
              "per 512-centroid pass) + hash_fixup_kernel (side stream) + the 3-product refinement of the rows the "
              "hi-only bound leaves")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=30)   # untimed; the step time settles over the first few dozen calls
    ap.add_argument("--n", type=int, default=10_000_000, help="points per GPU")
    ap.add_argument("--workload", choices=["c3", "c5"], default="c3")
    ap.add_argument("--k", type=int, default=None, help="centroids (default 256 for c3, 1024 for c5)")
    ap.add_argument("--no-c5", action="store_true", help="c3: leave out the C5 iteration object")
    ap.add_argument("--data", choices=["grid", "normal"], default="grid",
                    help="the rows: include/lshkm_synth.h's 2^-15 grid generator (default) or its full-mantissa "
                         "normal generator (SURVEY.md §8d)")
    ap.add_argument("--no-normal-leg", dest="normal_leg", action="store_false",
                    help="c3 on grid data: leave out the normal_data object (C3 + C5 on full-mantissa rows)")
    ap.add_argument("--recom-users", type=int, default=1024,
                    help="C5: query users per iteration of the recommend step (0: no recommend step)")
    ap.add_argument("--no-exact-dist-line", dest="exact_dist_line", action="store_false",
                    help="c3: leave out the timing with bit-exact (fp64 chain) distances")
    ap.add_argument("--dry-run", action="store_true", help="gloo on CPU, no GPU work (tests the rank plumbing)")
    ap.add_argument("--cpu-port-hash-sample", type=int, default=400_000)
    ap.add_argument("--cpu-port-assign-sample", type=int, default=300_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-hash-sample", type=int, default=100_000)
    ap.add_argument("--cpu-assign-sample", type=int, default=12_000)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-launch HBM bytes measured by rocprofv3 PMC passes (see profiles/)")
    ap.add_argument("--traffic-json-c5", default=os.path.join(ROOT, "profiles", "traffic_c5.json"))
    argv = json.loads(os.environ["LSHKM_BENCH_ARGV"]) if len(sys.argv) == 1 and "LSHKM_BENCH_ARGV" in os.environ \
        else sys.argv[1:]
    args = ap.parse_args(argv)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        return dry_run(args, world, rank)
    backend = "none (single process)"
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus
        backend = dist.get_backend()
        assert backend == "nccl", backend          # RCCL on ROCm
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    lk = load_pkg()
    ctx = lk.Context(local)
    lib = lk.lib()
    N = args.n
    N_total = N * world
    nb = N_total // BUCKET_DIV

    # Resident shard + parameters (untimed).
    X = ctx.synth(SEED_DATA, N, D, row0=rank * N, kind=args.data)
    V, t, r, _ = lk.params_lsh_euclidean(SEED_PARAMS, L_TABLES, K_FUNCS, D, W)
    lsh = lk.LSH(ctx, "euclidean", D, K_FUNCS, L_TABLES, nb, W, V=V, t=t, r=r)
    p = lambda t_: C.c_void_p(t_.data_ptr())

    def initial_centroids(K, kind):
        rows = sharding.centroid_rows(N_total, K)                  # reference init: rows i*floor(N/K)
        Cc = torch.empty((K, D), dtype=torch.float64, device=dev)
        for i, row in enumerate(rows):                             # centroids may live on other shards
            Cc[i] = ctx.synth(SEED_DATA, 1, D, row0=int(row), kind=kind)[0].double()
        return Cc, sharding.local_src_rows(rows, rank * N, N)      # centroid override, shard-local

    def c3_run(K, X=X, kind=args.data, steps=args.steps, warmup=args.warmup):
        Cc, src = initial_centroids(K, kind)
        tuples = torch.empty((N, L_TABLES, K_FUNCS), dtype=torch.int32, device=dev)
        bucket = torch.empty((N, L_TABLES), dtype=torch.int32, device=dev)
        assign = torch.empty((N,), dtype=torch.int32, device=dev)
        dist_ = torch.empty((N,), dtype=torch.float64, device=dev)
        src_p = src.ctypes.data_as(C.c_void_p)

        def step():
            # one pass: tuples + bucket IDs + cluster IDs + distances (lshkm_hash_assign)
            lk._ck(lib.lshkm_hash_assign(lsh.h, p(X), N, p(Cc), K, src_p, p(tuples), None, p(bucket), p(assign),
                                         p(dist_)))
        ctx.reset_stats()
        elapsed = timed(step, steps, warmup, world, dev)
        ex = {"per_step": True, "assign_ambiguous_rows": ctx.stat(lk.STAT_ASSIGN_AMBIG) // (steps + warmup),
              "hash_fixup_rows": ctx.stat(lk.STAT_HASH_FIX) // (steps + warmup),
              "hash_exact_fallbacks": ctx.stat(lk.STAT_HASH_EXACT) // (steps + warmup),
              "refined_rows": ctx.stat(lk.STAT_REFINED) // (steps + warmup)}
        kms = fused_kernel_ms(lk, lib, ctx, step, max(3, steps))
        if args.exact_dist_line:
            # the same step with every distance from the reference-order fp64 chain
            ctx.set_dist_mode("exact")
            try:
                ctx.reset_stats()
                el_x = timed(step, steps, warmup, world, dev)
                pow_fix = ctx.stat(lk.STAT_POW_FIX) // (steps + warmup)
                kms_x = fused_kernel_ms(lk, lib, ctx, step, max(3, steps))
            finally:
                ctx.set_dist_mode("certified")
            ex["exact_distances"] = {"note": "lshkm_ctx_set_dist_mode(LSHKM_DIST_EXACT): bit-exact distances "
                                             "(the reference's fp64 chain)",
                                     "value": N_total * steps / el_x, "ms_per_step": el_x / steps * 1e3,
                                     "kernel_ms": kms_x, "frac": 624.0 * N / (kms_x * 1e-3) / 8e12,
                                     "pow_fix_rows": pow_fix}
        return elapsed, kms, ex

    def c5_run(K, X=X, kind=args.data, steps=args.steps, warmup=args.warmup):
        # one full iteration: hash + assign, per-shard sums, RCCL all-reduce,
        # finalize, and the recommend step (get_top_N_recom over the whole
        # clusters of Q query users, the prediction sums carried rank to rank)
        Cc, src = initial_centroids(K, kind)
        it = sharding.ShardedLloyd(lk, ctx, lsh, X, Cc, src, mode="certified")
        if args.recom_users > 0:
            it.enable_recommend(N_total, rank * N, Q=args.recom_users, n_top=5)
        ctx.reset_stats()
        elapsed = timed(it.step, steps, warmup, world, dev)
        ex = {"per_step": True, "assign_ambiguous_rows": ctx.stat(lk.STAT_ASSIGN_AMBIG) // (steps + warmup),
              "hash_fixup_rows": ctx.stat(lk.STAT_HASH_FIX) // (steps + warmup),
              "refined_rows": ctx.stat(lk.STAT_REFINED) // (steps + warmup)}
        it.timing = True
        kms = fused_kernel_ms(lk, lib, ctx, it.step, max(3, steps))
        it.timing = False
        xms = it.exchange_ms()
        rec = None
        if args.recom_users > 0:
            it.recom_timing = []
            for _ in range(3):
                it.step()
            ph1 = sorted(a for a, _ in it.recom_timing)[1]
            ph2 = sorted(b for _, b in it.recom_timing)[1]
            it.recom_timing = None
            ucl = it.recom_ucl.cpu().numpy()
            counts = it.last_counts.cpu().numpy()
            sims = int(counts[ucl].sum())
            rec = {"what": "get_top_N_recom(neighbors, user, 5) over the user's whole cluster (crypto_rec.hpp:327-345, "
                           "main.cpp:260-269): x87-exact cosine similarities to every member and the "
                           "get_predicted_user_sim terms on every rank (lshkm_cluster_terms), then the prediction "
                           "sums carried rank to rank in row order (lshkm_cluster_chain_terms, RCCL point-to-point) "
                           "and the quicksort",
                   "users_per_step": args.recom_users, "n_top": 5,
                   "users": "rows i * floor(N_total / Q) of the whole job (their clusters span every shard)",
                   "similarities_per_step": sims, "sims_ms": ph1, "chain_ms": ph2,
                   "users_per_s": args.recom_users / ((ph1 + ph2) / 1e3),
                   "similarities_per_s": sims / ((ph1 + ph2) / 1e3)}
        rec = rec or {}
        rec["km_flagged_chains"] = it.flagged       # the last step's: carried rank to rank (segments)
        rec["exactness"] = ex
        return elapsed, kms, xms, rec

    def c5_object(K, elapsed, kms, xms, rec=None, steps=args.steps):
        coll = (f"sharding.kmeans_sums_sharded over RCCL ({backend}): all-gather of the {K}x128 fp64 partial sums, "
                f"all-reduces of the |x| sums, bit positions and {K} counts; the chains the global never-rounds "
                f"test flags carried rank to rank" if world > 1
                else "none (N = 1: a single shard, no collective)")
        return {
            "metric": f"C5 LSH-assign + k-means recommend iterations: points/s (hash + assign K={K} + sums + "
                      f"{'RCCL exchange' if world > 1 else 'no collective at N = 1'} + finalize"
                      + (f" + recommend for {args.recom_users} users)" if args.recom_users > 0 else ")"),
            "value": N_total * steps / elapsed, "unit": "point iteration ops/s",
            "ms_per_step": elapsed / steps * 1e3, "n_gpus": world, "scaling": "weak",
            "config": {"workload": f"C5 (BASELINE configs[4]): N={N} per GPU x {world} GPU(s), d=128, K={K}, "
                                   f"L=5, k=4, w=0.4, exchange: {coll}",
                       "N_per_gpu": N, "N_total": N_total, "K": K, "parallelism": f"dp{world} (row shards)"},
            "allreduce": coll,
            "km_sums_exchange_ms": xms,         # the sums + their exchange + certificate (HIP events)
            "km_flagged_chains": (rec or {}).pop("km_flagged_chains", None),
            "exactness": (rec or {}).pop("exactness", None),
            "recommend": rec or None,
            "roofline": roofline(N, K, kms, traffic_for(args.traffic_json_c5, N, K, "c5"),
                                 FUSED_WHAT + " (K = 1024: two 512-centroid passes)"),
        }

    line = None
    if args.workload == "c5":
        K = args.k or 1024
        el, kms, xms, rec = c5_run(K)
        line = c5_object(K, el, kms, xms, rec)
        line.update({"metric": METRIC + " (C5 workload)", "unit": "point hash+assign ops/s", "steps": args.steps,
                     "warmup": args.warmup, "higher_is_better": True, "vs_baseline": None,
                     "dtype": DTYPE,
                     "data": DATA[args.data]})
    else:
        K = args.k or 256
        el, kms, ex = c3_run(K)
        line = {
            "metric": METRIC, "value": N_total * args.steps / el, "unit": "point hash+assign ops/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": DTYPE,
            "data": DATA[args.data],
            "config": {"workload": f"C3 Lloyd K={K} + C2 LSH L=5 k=4 hashing, N={N} per GPU, d=128",
                       "N_per_gpu": N, "N_total": N_total, "d": D, "K": K, "L": L_TABLES, "k": K_FUNCS,
                       "w": W, "nb": nb, "parallelism": f"dp{world} (row shards)"},
            "roofline": roofline(N, K, kms, traffic_for(args.traffic_json, N, K, "c3"), FUSED_WHAT),
            "exactness": ex,
        }
        if not args.no_c5:
            K5 = 1024
            el5, kms5, xms5, rec5 = c5_run(K5)
            line["c5"] = c5_object(K5, el5, kms5, xms5, rec5)
        if args.data == "grid" and args.normal_leg:
            # the same C3 step and C5 iteration on full-mantissa rows (SURVEY.md
            # §8d's N(0,1) data): the certificates' and exact chains' rates there
            Xn = ctx.synth(SEED_DATA, N, D, row0=rank * N, kind="normal")
            ns, nw = max(5, args.steps // 2), max(5, args.warmup // 3)
            el_n, kms_n, ex_n = c3_run(K, X=Xn, kind="normal", steps=ns, warmup=nw)
            nd = {"data": DATA["normal"], "steps": ns, "warmup": nw,
                  "c3": {"value": N_total * ns / el_n, "ms_per_step": el_n / ns * 1e3, "kernel_ms": kms_n,
                         "frac": BYTES_PER_PT * N / (kms_n * 1e-3) / (HBM_PEAK_GBS * 1e9), "exactness": ex_n}}
            if not args.no_c5:
                el5, kms5, xms5, rec5 = c5_run(1024, X=Xn, kind="normal", steps=ns, warmup=nw)
                nd["c5"] = c5_object(1024, el5, kms5, xms5, rec5, steps=ns)
                nd["c5"].pop("roofline")
                nd["c5"]["kernel_ms"] = kms5
            line["normal_data"] = nd
    line["world_size"] = world
    line["backend"] = backend
    if world > 1:
        torch.distributed.barrier()       # every rank's timed work is done before the CPU baseline runs
    if rank == 0 and not args.no_cpu_baseline:
        # the reference's CPU path on this host, in the same run (rank 0 only; at
        # N > 1 after the final barrier, so no rank's timing overlaps it)
        attach_cpu_baseline(line, args, line["config"]["K"])
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
