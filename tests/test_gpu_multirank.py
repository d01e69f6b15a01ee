"""The multi-rank product path on the GPU: two fresh processes
share the one MI355X over gloo, each running liblshkm on its row shard
(tests/mr_worker.py), against one process over all rows.

  - hash tuples, bucket IDs, cluster IDs and distances: bit-exact (per row),
    in both distance modes of the context (certified: the shipped default;
    exact), and the iteration-0 distances against the oracle per the mode;
  - k-means centers, fast mode (all-reduce of per-shard sums): <= 1e-13 rel;
  - k-means centers, exact mode (rank-to-rank carry chain): bit-exact;
  - cosine (cosine index + cosine Lloyd in one pass, fast mode): buckets,
    IDs, distances bit-exact, centers <= 1e-13 rel;
  - sharded euclidean hypercube: the same coins (global first-occurrence
    order) and vertices as the single-process build.
K = 1024 with hashing: the per-shard step is C5's kernel form.
The C5 bench line (bench.py --workload c5) runs the same ShardedLloyd step."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "mr_worker.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, out, dist_mode):
    port = str(_free_port())
    env = {k: v for k, v in os.environ.items() if k != "LSHKM_DIST"}      # the ABI mode alone decides
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    procs = [subprocess.Popen([sys.executable, "-u", WORKER, str(r), str(world), port, str(out), dist_mode], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    return [dict(np.load(os.path.join(out, f"rank{r}.npz"))) for r in range(world)]


@pytest.mark.parametrize("dist_mode", ["certified", "exact"])
def test_two_ranks_on_one_gpu_match_single_process(tmp_path, dist_mode):
    (tmp_path / "one").mkdir()
    (tmp_path / "two").mkdir()
    one = _run(1, tmp_path / "one", dist_mode)[0]
    two = _run(2, tmp_path / "two", dist_mode)
    assert all(str(r["dist_mode"][0]) == dist_mode for r in two + [one])
    cat = lambda key: np.concatenate([r[key] for r in two])
    for mode in ("fast", "exact"):
        assert np.array_equal(cat(f"{mode}_tuples"), one[f"{mode}_tuples"]), mode
        assert np.array_equal(cat(f"{mode}_bucket"), one[f"{mode}_bucket"]), mode
    # iteration 0 runs on the same dataset-row centroids everywhere: bit-exact
    for mode in ("fast", "exact"):
        assert np.array_equal(cat(f"{mode}_assign0"), one[f"{mode}_assign0"]), mode
        assert np.array_equal(cat(f"{mode}_dist0").view(np.uint64), one[f"{mode}_dist0"].view(np.uint64)), mode
    # exact mode: the carry chain reproduces the single pass bit for bit, so
    # every later iteration is identical too
    for s in range(2):
        assert np.array_equal(cat(f"exact_assign{s}"), one[f"exact_assign{s}"]), s
        for r in two:
            assert np.array_equal(r[f"exact_centers{s + 1}"].view(np.uint64),
                                  one[f"exact_centers{s + 1}"].view(np.uint64)), s
    # fast mode: sums reassociate across the all-reduce
    c1, c1_one = two[0]["fast_centers1"], one["fast_centers1"]
    assert np.array_equal(c1, two[1]["fast_centers1"])       # every rank holds the same centers
    rel = np.abs(c1 - c1_one) / np.maximum(np.abs(c1_one), 1e-300)
    assert rel.max() <= 1e-13
    # cosine iteration: per-row outputs bit-exact, centers within the fast-mode bound
    for key in ("cos_bucket", "cos_assign0"):
        assert np.array_equal(cat(key), one[key]), key
    assert np.array_equal(cat("cos_dist0").view(np.uint64), one["cos_dist0"].view(np.uint64))
    cc, cc_one = two[0]["cos_centers1"], one["cos_centers1"]
    assert np.array_equal(cc, two[1]["cos_centers1"])
    assert (np.abs(cc - cc_one) / np.maximum(np.abs(cc_one), 1e-300)).max() <= 1e-13
    # iteration 0 against the oracle: IDs bit-exact, distances per the mode's
    # contract (a sample of rows; centroid-override rows are (c, 0))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from conftest import assert_dist
    sys.path.insert(0, os.path.join(ROOT, "crypto-recommendation_amd"))
    import sharding as sh
    N, K = 120_000, 1024
    rows = sh.centroid_rows(N, K)
    Xall = oracle.synth(0x5EED, N, 128)
    sub = np.setdiff1d(np.random.default_rng(8).choice(N, 2000, replace=False), rows)
    oa, od = oracle.lloyd_assign(Xall[sub], Xall[rows].astype(np.float64), "euclidean", None)
    assert np.array_equal(cat("fast_assign0")[sub], oa)
    assert_dist(cat("fast_dist0")[sub], od, dist_mode)
    # the C5 recommend step (recommend_sharded: the prediction sums carried from
    # rank to rank): every rank holds the single process's result, which is the
    # oracle's get_top_N_recom over the users' whole clusters
    for s in range(2):
        for r in two:
            assert np.array_equal(r[f"recom_ucl{s}"], one[f"recom_ucl{s}"]), s
            assert np.array_equal(r[f"recom{s}"], one[f"recom{s}"]), s
    qrows = np.arange(96, dtype=np.int64) * (N // 96)
    sets = [np.nonzero((7 * np.arange(128) + int(r)) % 16 == 0)[0].astype(np.int32) for r in qrows]
    up = np.cumsum([0] + [len(x) for x in sets]).astype(np.int64)
    crow, crows = oracle.clusters_csr(one["fast_assign1"], K)
    want = oracle.cluster_top_n(Xall, np.zeros(N), crow, crows, Xall[qrows], np.zeros(96), one["recom_ucl1"], up,
                                np.concatenate(sets), 5)
    assert np.array_equal(one["recom_ucl1"], one["fast_assign1"][qrows])
    assert np.array_equal(one["recom1"], want)
    # hypercube: same coins, same engine state, same vertices
    for key in ("memo_f", "memo_h", "memo_bit", "memo_state"):
        for r in two:
            assert np.array_equal(r[key], one[key]), key
    assert np.array_equal(cat("vertex"), one["vertex"])
