"""Timings of the SURVEY §8 rows beside the headline (one MI355X): each row's
device call at a production-like size, inputs resident in HBM: "gpu_s" is the
time per call with calls back to back (HIP events on the library's stream, as
bench.py times its steps), "call_s" the median of single calls between host
syncs (host launch and sync latency included) -- next to the CPU restatement (oracle/, one
thread, OMP_NUM_THREADS=1, kind "port") on a bounded sample of the same
workload, scaled to the row's unit. Prints one JSON line per row.

    python tools/bench_rows.py [--rows cosine,kpp,range,sil,update,lsh,cube,recom,csv,f64] [--no-cpu]
"""
import argparse
import json
import os
import sys
import tempfile
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from amd import lshkm  # noqa: E402


class GpuTime(float):
    """Seconds per call, back to back (HIP events on the library's stream around
    reps calls, as bench.py times its steps); .call: the median of single calls
    each bracketed by host syncs (host launch and sync latency included)."""
    call = None


def gpu_time(ctx, fn, reps=5):
    fn()
    ctx.sync()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        ctx.sync()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    ctx.sync()
    torch.cuda.synchronize()
    t = GpuTime(e0.elapsed_time(e1) / 1e3 / reps)
    t.call = float(np.median(ts))
    t.calls = 2 * reps + 1          # fn's calls here (stat counters divide by it)
    return t


def cpu_time(fn):
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md


def emit(row, unit, units, t_gpu, cpu=None, note="", bytes_per_unit=None):
    line = {"row": row, "unit": unit, "units": units, "gpu_s": float(t_gpu), "gpu_rate": units / t_gpu}
    if getattr(t_gpu, "call", None) is not None:
        line["call_s"] = t_gpu.call          # one call between host syncs
    if bytes_per_unit:
        # algorithmic HBM bytes of the whole call (stated per unit) over its time per call
        gbs = units * bytes_per_unit / t_gpu / 1e9
        line["roofline"] = {"bound": "hbm", "bytes_per_unit": bytes_per_unit, "achieved": gbs,
                            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS}
    if cpu:
        cu, ct, sample = cpu
        line["cpu_baseline"] = {"rate": cu / ct, "kind": "port", "cores": 1, "sample": sample}
        line["gpu_over_cpu"] = line["gpu_rate"] / line["cpu_baseline"]["rate"]
    if note:
        line["note"] = note
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="cosine,kpp,range,sil,update,lsh,cube,recom,csv,f64")
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    rows = set(a.rows.split(","))
    ctx = lshkm.Context(0)
    cpu = not a.no_cpu

    if "update" in rows:     # k_means (update.hpp:37-86), exact-order sums, C3 shape
        N, d, K = 10_000_000, 128, 256
        X = ctx.synth(0x5EED, N, d)
        src = (np.arange(K) * (N // K)).astype(np.int64)
        C = X[torch.from_numpy(src).to(ctx.dev)].double()
        asg, _ = lshkm.lloyd_assign(ctx, X, C, "euclidean", src.astype(np.int32))
        t = gpu_time(ctx, lambda: lshkm.kmeans_update(ctx, X, asg, C, "euclidean", 0.05))
        c = None
        if cpu:
            n = 1_000_000
            Xh, ah = X[:n].cpu().numpy(), asg[:n].cpu().numpy()
            c = (n, cpu_time(lambda: oracle.kmeans_update(Xh, ah, C.cpu().numpy(), "euclidean", 0.05)),
                 f"{n} rows, K={K}, d={d}")
        emit("k_means update", "rows/s", N, t, c, "N=10M, d=128, K=256; bytes: the row + its cluster id",
             bytes_per_unit=4 * d + 4)
        del X

    if "cosine" in rows:     # lloyds_assignment, cosine metric (assignment.hpp:52-75)
        N, d, K = 10_000_000, 128, 256
        X = ctx.synth(0x5EED + 4, N, d)
        src = (np.arange(K) * (N // K)).astype(np.int64)
        C = X[torch.from_numpy(src).to(ctx.dev)].double()
        ctx.reset_stats()
        t = gpu_time(ctx, lambda: lshkm.lloyd_assign(ctx, X, C, "cosine"))
        amb = ctx.stat(lshkm.STAT_ASSIGN_AMBIG) / t.calls
        cfix = ctx.stat(lshkm.STAT_COS_FIX) / t.calls
        os.environ["LSHKM_ASSIGN_PATH"] = "exact"
        te = gpu_time(ctx, lambda: lshkm.lloyd_assign(ctx, X, C, "cosine"), reps=1)
        del os.environ["LSHKM_ASSIGN_PATH"]
        c = None
        if cpu:
            n = 20_000
            Xh = X[:n].cpu().numpy()
            c = (n, cpu_time(lambda: oracle.lloyd_assign(Xh, C.cpu().numpy(), "cosine", None)), f"{n} rows, K={K}")
        emit("lloyds_assignment (cosine)", "rows/s", N, t, c,
             f"N=10M, d=128, K=256; hi-only f16 kernel (normalised centroids), {amb:.0f} rows/call to the pruned exact "
             f"pass, {cfix:.0f} winner distances/call to the soft-x87 chain; "
             f"exact all-K pass alone {te * 1e3:.1f} ms; bytes: the row + cluster id and distance",
             bytes_per_unit=4 * d + 12)
        # main.cpp's cosine flow in one pass: CosineGGen buckets (L=5, k=4) + cosine Lloyd
        R, _ = lshkm.params_lsh_cosine(12345, 5, 4, d)
        lsh = lshkm.LSH(ctx, "cosine", d, 4, 5, R=R)
        th = gpu_time(ctx, lambda: lshkm.hash_assign(lsh, X, C, tuples=False, bucket=True, metric="cosine"))
        tsep = gpu_time(ctx, lambda: (lsh.hash(X, tuples=False, phi=False), lshkm.lloyd_assign(ctx, X, C, "cosine")))
        emit("hash_assign (cosine LSH + cosine Lloyd)", "rows/s", N, th, None,
             f"N=10M, d=128, L=5, k=4, K=256, one pass (lshkm_hash_assign_metric); the two separate calls "
             f"{tsep * 1e3:.2f} ms; bytes: the row + cluster id, distance and 5 bucket ids",
             bytes_per_unit=4 * d + 12 + 4 * 5)
        del X

    if "kpp" in rows:        # k_means_pp (initialization.hpp:71-156)
        N, d, K = 1_000_000, 128, 64
        X = ctx.synth(0x5EED + 1, N, d)
        t = gpu_time(ctx, lambda: lshkm.kmeans_pp_rows(ctx, X, K, "euclidean", 7), reps=3)
        c = None
        if cpu:
            n = 100_000
            Xh = X[:n].cpu().numpy()
            c = (n * K, cpu_time(lambda: oracle.kmeans_pp(Xh, K, "euclidean", 7)), f"{n} rows, K={K}")
        emit("k_means_pp", "row-centroid steps/s", N * K, t, c,
             "N=1M, d=128, K=64, euclidean; bytes: one pass over the rows and D^2 per centroid",
             bytes_per_unit=4 * d + 8)
        del X

    if "range" in rows:      # lsh_range_assignment (assignment.hpp:108-217)
        N, d, K, L, k = 1_000_000, 128, 256, 5, 4
        X = ctx.synth(0x5EED + 2, N, d)
        V, tt, r, _ = lshkm.params_lsh_euclidean(77, L, k, d, 4.0)
        lsh = lshkm.LSH(ctx, "euclidean", d, k, L, N // 100, 4.0, V=V, t=tt, r=r)
        lsh.build(X)
        src = (np.arange(K) * (N // K)).astype(np.int32)
        Q = X[torch.from_numpy(src.astype(np.int64)).to(ctx.dev)]
        C = Q.double()

        def run():
            ptr, ci = lsh.query(Q, filtered=False, device=True)
            return lshkm.range_assign(ctx, X, C, ptr, ci, "euclidean", src_rows=src)
        t = gpu_time(ctx, run, reps=3)
        c = None
        if cpu:
            n = 100_000
            Xs = X[:n].contiguous()
            lsh2 = lshkm.LSH(ctx, "euclidean", d, k, L, n // 100, 4.0, V=V, t=tt, r=r)
            lsh2.build(Xs)
            s2 = (np.arange(K) * (n // K)).astype(np.int32)
            Q2 = Xs[torch.from_numpy(s2.astype(np.int64)).to(ctx.dev)]
            p2, c2 = lsh2.query(Q2, filtered=False)
            Xh, C2 = Xs.cpu().numpy(), Q2.double().cpu().numpy()
            c = (n, cpu_time(lambda: oracle.range_assign(Xh, C2, p2, c2, "euclidean", src_rows=s2)), f"{n} rows, K={K}")
        emit("lsh_range_assignment", "rows/s", N, t, c, "N=1M, d=128, K=256, L=5, k=4, w=4 (query + range + Lloyd rest)")
        del X

    if "sil" in rows:        # silhouette_cluster (silhouette.hpp:31-144)
        N, d, K = 100_000, 128, 16
        X = ctx.synth(0x5EED + 3, N, d)
        src = (np.arange(K) * (N // K)).astype(np.int64)
        C = X[torch.from_numpy(src).to(ctx.dev)].double()
        asg, _ = lshkm.lloyd_assign(ctx, X, C, "euclidean", src.astype(np.int32))
        pairs = float(np.sum(np.bincount(asg.cpu().numpy(), minlength=K).astype(np.float64) ** 2) * 2)
        t = gpu_time(ctx, lambda: lshkm.silhouette(ctx, X, asg, C, "euclidean"), reps=3)
        c = None
        if cpu:
            n = 10_000
            Xh = X[:n].cpu().numpy()
            ah, _ = oracle.lloyd_assign(Xh, C.cpu().numpy(), "euclidean", None)
            p2 = float(np.sum(np.bincount(ah, minlength=K).astype(np.float64) ** 2) * 2)
            c = (p2, cpu_time(lambda: oracle.silhouette(Xh, ah, C.cpu().numpy(), "euclidean")), f"{n} rows, K={K}")
        emit("silhouette_cluster", "distance pairs/s", pairs, t, c, "N=100k, d=128, K=16")
        del X

    if "lsh" in rows:        # create_LSH_hashtables + get_LSH_filtered_combined_buckets (C2)
        N, d, L, k = 1_000_000, 128, 5, 4
        X = ctx.synth(0x5EED, N, d)
        V, tt, r, _ = lshkm.params_lsh_euclidean(12345, L, k, d, 0.4)
        lsh = lshkm.LSH(ctx, "euclidean", d, k, L, N // 100, 0.4, V=V, t=tt, r=r)
        tb = gpu_time(ctx, lambda: lsh.build(X))
        c = None
        if cpu:
            n = 200_000
            Xh = X[:n].cpu().numpy()
            c = (n, cpu_time(lambda: oracle.bucket_csr(oracle.lsh_hash_euclid(Xh, V, tt, np.float32(0.4), r, N // 100)[2],
                                                       N // 100)), f"{n} rows")
        emit("create_LSH_hashtables", "rows/s", N, tb, c,
             "C2: N=1M, d=128, L=5, k=4, w=0.4, nb=10k; bytes: the row + per table its bucket key and CSR slot",
             bytes_per_unit=4 * d + 5 * 8)
        nq = 65_536
        qrows = torch.arange(nq, device=ctx.dev) * (N // nq)
        Q = X[qrows]
        alias = qrows.to(torch.int32)
        tq = gpu_time(ctx, lambda: lsh.query(Q, True, alias, device=True))
        tot = int(lsh.query(Q, True, alias, device=True)[0][-1])
        emit("get_LSH_filtered_combined_buckets", "queries/s", nq, tq, None,
             f"65,536 dataset-row queries, C2 index; {tot} rows returned",)
        del X

    if "cube" in rows:       # create_hypercube + get_hypercube_combined_buckets (C4)
        N, d, k = 10_000_000, 128, 14
        X = ctx.synth(0x5EED, N, d)
        V, tt, st = lshkm.params_cube_euclidean(4242, k, d, 2.0)
        cubes = []

        def fresh_build():        # create_hypercube: new generators, an empty coin memo
            c = lshkm.Cube(ctx, "euclidean", d, k, 2.0, V=V, t=tt, rng_state=st)
            c.build(X)
            cubes.append(c)
        tb = gpu_time(ctx, fresh_build, reps=3)
        cube = cubes[-1]
        tr = gpu_time(ctx, lambda: cube.build(X), reps=3)
        emit("create_hypercube", "rows/s", N, tb, None,
             f"C4: N=10M, d=128, d'=14, w=2 (euclidean F coins), fresh cube each build; "
             f"rebuild with the coins already drawn {tr * 1e3:.2f} ms; bytes: the row + its vertex and CSR slot",
             bytes_per_unit=4 * d + 8)
        nq = 65_536
        Q = X[torch.arange(nq, device=ctx.dev) * (N // nq)]
        tq = gpu_time(ctx, lambda: cube.query(Q, 14, device=True), reps=3)
        tot = int(cube.query(Q, 14, device=True)[0][-1])
        emit("get_hypercube_combined_buckets", "queries/s", nq, tq, None,
             f"65,536 queries, probes=14 (Hamming<=1); {tot} candidate rows returned (bytes: 4 B read + 4 B "
             f"written per candidate)", bytes_per_unit=8.0 * tot / nq)
        del X

    if "recom" in rows:      # get_P_closest + get_top_N_recom (crypto_rec.hpp:213-325)
        N, d, Q, P, NT = 200_000, 100, 20_000, 20, 5
        rng = np.random.default_rng(5)
        Xh = rng.integers(-40, 41, size=(N, d)).astype(np.float64) / 8.0
        X = torch.from_numpy(Xh).to(ctx.dev)
        Uh = Xh[rng.integers(0, N, Q)]
        U = torch.from_numpy(Uh).to(ctx.dev)
        cand = [np.sort(rng.choice(N, 200, replace=False)).astype(np.int32) for _ in range(Q)]
        cp = torch.from_numpy(np.cumsum([0] + [len(c) for c in cand]).astype(np.int64)).to(ctx.dev)
        ci = torch.from_numpy(np.concatenate(cand)).to(ctx.dev)
        t = gpu_time(ctx, lambda: lshkm.p_closest(ctx, X, U, cp, ci, P))
        c = None
        if cpu:
            q2 = 2000
            cph, cih = cp[:q2 + 1].cpu().numpy(), ci[:int(cp[q2])].cpu().numpy()
            c = (q2, cpu_time(lambda: oracle.p_closest(Xh, Uh[:q2], cph, cih, P)), f"{q2} users x 200 candidates")
        emit("get_P_closest", "users/s", Q, t, c, f"N={N}, d={d}, {Q} users x 200 candidates, P={P}")

    if "f64" in rows:        # the reference's own shapes: fp64 user vectors, d = number of coins
        # (main.cpp:149-222 cosine LSH recommend, :240-281 clustering recommend; crypto_rec.hpp:78-140)
        # main.cpp:155-168: every user queries the cosine index over all users
        # (k = 4: a bucket holds ~N/16 users per table, so the work grows as N^2)
        N, d, P, NT = 20_000, 100, 20, 5
        rng = np.random.default_rng(11)
        Xh = rng.standard_normal((N, d))                  # general doubles: the _f64 entry points
        X = torch.from_numpy(Xh).to(ctx.dev)
        R, _ = lshkm.params_lsh_cosine(12345, 5, 4, d)
        lsh = lshkm.LSH(ctx, "cosine", d, 4, 5, R=R)
        tb = gpu_time(ctx, lambda: lsh.build(X))
        emit("create_LSH_hashtables (cosine, fp64 rows)", "rows/s", N, tb, None,
             f"N={N}, d={d} fp64 user vectors, L=5, k=4 (main.cpp:155); bytes: the fp64 row + per table its "
             f"bucket key and CSR slot", bytes_per_unit=8 * d + 5 * 8)
        nq = N
        qrows = torch.arange(nq, device=ctx.dev)
        Q = X[qrows]
        alias = qrows.to(torch.int32)
        tq = gpu_time(ctx, lambda: lsh.query(Q, True, alias, device=True), reps=3)
        cptr, cidx = lsh.query(Q, True, alias, device=True)
        tot = int(cptr[-1])
        emit("get_LSH_filtered_combined_buckets (cosine, fp64 rows)", "queries/s", nq, tq, None,
             f"every user of N={N} as a query; {tot} candidate rows ({tot / nq:.0f} per query); bytes: 4 B "
             f"read + 4 B written per candidate", bytes_per_unit=8.0 * tot / nq)
        tp = gpu_time(ctx, lambda: lshkm.p_closest(ctx, X, Q, cptr, cidx, P), reps=3)
        emit("get_P_closest (fp64 rows)", "candidates/s", tot, tp, None,
             f"{nq} users x {tot / nq:.0f} candidates, d={d}, P={P}; bytes: the candidate's fp64 row (the {N} rows "
             f"fit the Infinity Cache: L2/MALL bandwidth, not HBM)", bytes_per_unit=8 * d + 4)
        idx, sim, cnt = lshkm.p_closest(ctx, X, Q, cptr, cidx, P)
        xm = X.mean(dim=1).contiguous()
        um = xm[qrows].contiguous()
        unk = [np.sort(rng.choice(d, 20, replace=False)).astype(np.int32) for _ in range(nq)]
        up = torch.from_numpy(np.arange(nq + 1, dtype=np.int64) * 20).to(ctx.dev)
        ui = torch.from_numpy(np.concatenate(unk)).to(ctx.dev)
        tn = gpu_time(ctx, lambda: lshkm.top_n_recom(ctx, X, xm, um, up, ui, idx, sim, cnt, NT), reps=3)
        emit("get_top_N_recom (fp64 rows)", "users/s", nq, tn, None, f"{nq} users, P={P}, 20 unknown coins each, N={NT}")
        del lsh, cptr, cidx, X
        # clustering recommendation's Lloyd + k_means on fp64 user vectors (main.cpp:248-258), at 1M users
        N, K = 1_000_000, 256
        X = torch.from_numpy(rng.standard_normal((N, d))).to(ctx.dev)
        src = (np.arange(K) * (N // K)).astype(np.int64)
        C = X[torch.from_numpy(src).to(ctx.dev)].clone()
        for metric in ("euclidean", "cosine"):
            ctx.reset_stats()
            t = gpu_time(ctx, lambda: lshkm.lloyd_assign(ctx, X, C, metric))
            amb = ctx.stat(lshkm.STAT_ASSIGN_AMBIG) / t.calls
            emit(f"lloyds_assignment ({metric}, fp64 rows)", "rows/s", N, t, None,
                 f"N={N}, d={d} fp64, K={K}; {amb:.0f} rows/call to the exact pass; bytes: the fp64 row + id and "
                 f"distance", bytes_per_unit=8 * d + 12)
        asg, _ = lshkm.lloyd_assign(ctx, X, C, "euclidean")
        t = gpu_time(ctx, lambda: lshkm.kmeans_update(ctx, X, asg, C, "euclidean", 0.05))
        emit("k_means update (fp64 rows)", "rows/s", N, t, None, f"N={N}, d={d} fp64, K={K}; bytes: the fp64 row + id",
             bytes_per_unit=8 * d + 4)
        del X

    if "csv" in rows:        # VectorReader (vector_reader.hpp:54-85)
        n, d = 200_000, 64
        Xh = np.random.default_rng(9).standard_normal((n, d)).astype(np.float32)
        with tempfile.NamedTemporaryFile("w", suffix=".csv", delete=False) as f:
            for i in range(n):
                f.write(f"{i}," + ",".join(repr(float(v)) for v in Xh[i]) + "\n")
            path = f.name
        mb = os.path.getsize(path) / 1e6
        t0 = time.perf_counter(); lshkm.read_vectors(path, ",", 1, 0); t = time.perf_counter() - t0
        t1 = time.perf_counter(); lshkm.read_vectors(path, ",", 1, 1); t1 = time.perf_counter() - t1
        os.unlink(path)
        emit("VectorReader::read", "MB/s", mb, t, (mb, t1, f"{mb:.0f} MB, 1 thread of the same parser"),
             f"{n} x {d} CSV, all host threads (host-side row)")


if __name__ == "__main__":
    main()
