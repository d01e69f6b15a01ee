"""The reference's clustering driver for the project-2 vectors (main.cpp:81-111,
BASELINE.json configs[0] "C1"), on the MI355X path:

    cluster.conf -> get_config (lshkm_config_load)
    proj_2_input -> VectorReader<double>::read (lshkm_vectors_read)
    k_means_pp (cosine) -> while (continue && it < max_algo_iterations):
        lloyds_assignment; continue = k_means(min_dist_kmeans)

Host orchestration in Python over the C ABI (the reference's main is host
code too); every step runs in liblshkm. Rows go to the device as fp32 when
every value is an fp32 value (the tuned storage) and as fp64 otherwise (the
`_f64` entry points: the proj-2 CSV is parsed with stod, vector_reader.hpp:75-77,
so general doubles are the normal case); the results are the same either way.
"""
import os

import numpy as np

from lshkm import LshkmError, kmeans_pp_rows, kmeans_update, lloyd_assign, load_config, read_vectors


def device_rows(ctx, X_host):
    """Rows on the device: fp32 if every value (NaN payloads included) survives
    the round trip, else fp64."""
    X64 = np.ascontiguousarray(X_host, np.float64)
    X32 = X64.astype(np.float32)
    exact = np.array_equal(X32.astype(np.float64).view(np.uint64), X64.view(np.uint64))
    return ctx.torch.from_numpy(X32 if exact else X64).to(ctx.dev)


def cluster_vectors(ctx, X_host, K, max_iters, min_dist, seed, metric="cosine"):
    """k-means++ + Lloyd + k-means (main.cpp:94-111).
    Returns dict(rows, assign, dist, centers, iters, cont) (numpy)."""
    torch = ctx.torch
    X = device_rows(ctx, X_host)
    rows = kmeans_pp_rows(ctx, X, K, metric, seed)
    C = X[torch.from_numpy(rows.astype(np.int64)).to(ctx.dev)].double()
    src = rows            # initial centroids are dataset rows: the override applies (assignment.hpp:77-78)
    it, cont = 0, True
    assign = dist = None
    while cont and it < max_iters:
        assign, dist = lloyd_assign(ctx, X, C, metric, src)
        Cn, _, cont = kmeans_update(ctx, X, assign, C, metric, min_dist)
        if cont:          # k_means replaces every center (update.hpp:70-79)
            C, src = Cn, None
        it += 1
    ctx.sync()
    return dict(rows=rows, assign=assign.cpu().numpy(), dist=dist.cpu().numpy(), centers=C.cpu().numpy(),
                iters=it, cont=cont)


def run_proj2(ctx, config_path, seed, csv_path=None):
    """main.cpp:81-111 driven by cluster.conf. csv_path overrides proj_2_input."""
    c = load_config(config_path)
    path = csv_path or c.proj_2_input.decode()
    if not os.path.isabs(path):
        path = os.path.join(os.path.dirname(os.path.abspath(config_path)), path)
    ids, X, _, _ = read_vectors(path, c.proj_2_csv_delimiter.decode(), 1)
    if len(ids) == 0:
        raise LshkmError("no input vectors")     # main.cpp:87-89 returns -1
    res = cluster_vectors(ctx, X, c.proj_2_cluster_num, c.max_algo_iterations, c.min_dist_kmeans, seed)
    res["ids"] = ids
    return res
