"""The multi-rank product path on the GPU: two fresh processes
share the one MI355X over gloo, each running liblshkm on its row shard
(tests/mr_worker.py), against one process over all rows.

  - hash tuples, bucket IDs, cluster IDs and distances: bit-exact (per row),
    in both distance modes of the context (certified: the shipped default;
    exact), and the iteration-0 distances against the oracle per the mode;
  - k-means centers, both update modes -- "certified" (kmeans_sums_sharded:
    all-gather + all-reduces, the global never-rounds test, only the flagged
    chains carried) and "carry" (every chain carried rank to rank) --
    bit-exact over 3 iterations, on the grid rows at K = 1024 and on general
    rows: full-mantissa fp32, fp32 of a wide dynamic range (rounding chains:
    the carry runs) and fp64 doubles (segment records, composition in rank
    order); the single process's first update against the oracle;
  - cosine (cosine index + cosine Lloyd in one pass): buckets, IDs,
    distances and centers bit-exact;
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
    bits = lambda a: np.ascontiguousarray(a).view(np.uint64)
    for mode in ("certified", "carry"):
        assert np.array_equal(cat(f"{mode}_tuples"), one[f"{mode}_tuples"]), mode
        assert np.array_equal(cat(f"{mode}_bucket"), one[f"{mode}_bucket"]), mode
    # iteration 0 runs on the same dataset-row centroids everywhere: bit-exact
    for mode in ("certified", "carry"):
        assert np.array_equal(cat(f"{mode}_dist0").view(np.uint64), one[f"{mode}_dist0"].view(np.uint64)), mode
    # both update modes reproduce the single pass bit for bit, so every later
    # iteration is identical too; every rank holds the same centers
    for s in range(3):
        for mode in ("certified", "carry"):
            assert np.array_equal(cat(f"{mode}_assign{s}"), one[f"{mode}_assign{s}"]), (mode, s)
            for r in two:
                assert np.array_equal(bits(r[f"{mode}_centers{s + 1}"]), bits(one[f"{mode}_centers{s + 1}"])), (mode, s)
        assert np.array_equal(bits(one[f"certified_centers{s + 1}"]), bits(one[f"carry_centers{s + 1}"])), s
    # general rows: 3 iterations, both modes, two ranks == one process == each other
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    for leg in ("normal", "wide", "f64"):
        for s in range(3):
            for mode in ("certified", "carry"):
                assert np.array_equal(cat(f"{leg}_{mode}_assign{s}"), one[f"{leg}_{mode}_assign{s}"]), (leg, mode, s)
                for r in two:
                    assert np.array_equal(bits(r[f"{leg}_{mode}_centers{s + 1}"]),
                                          bits(one[f"{leg}_{mode}_centers{s + 1}"])), (leg, mode, s)
                    assert r[f"{leg}_{mode}_cont{s}"][0] == one[f"{leg}_{mode}_cont{s}"][0]
            assert np.array_equal(bits(one[f"{leg}_certified_centers{s + 1}"]),
                                  bits(one[f"{leg}_carry_centers{s + 1}"])), (leg, s)
            assert two[0][f"{leg}_flagged{s}"][0] == two[1][f"{leg}_flagged{s}"][0]     # the same test on every rank
    # the rounding chains were exercised: the wide fp32 and the fp64 legs flag chains
    assert two[0]["wide_flagged0"][0] > 0 and two[0]["f64_flagged0"][0] > 0
    # the single process's first update of each general leg against the oracle
    N = 120_000
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import mr_worker
    for leg, Kg in (("normal", 64), ("wide", 48), ("f64", 32)):
        Xf = oracle.synth(0x5EED, N, 128, kind="normal") if leg == "normal" else mr_worker.general_rows(leg, 0, N)
        grows = (np.arange(Kg) * (N // Kg)).astype(np.int64)
        Co, _, _ = oracle.kmeans_update(Xf, one[f"{leg}_certified_assign0"], Xf[grows].astype(np.float64),
                                        "euclidean", 0.0)
        assert np.array_equal(bits(one[f"{leg}_certified_centers1"]), bits(Co)), leg
    # cosine iteration: per-row outputs and centers bit-exact
    for key in ("cos_bucket", "cos_assign0"):
        assert np.array_equal(cat(key), one[key]), key
    assert np.array_equal(cat("cos_dist0").view(np.uint64), one["cos_dist0"].view(np.uint64))
    for r in two:
        assert np.array_equal(bits(r["cos_centers1"]), bits(one["cos_centers1"]))
    # iteration 0 against the oracle: IDs bit-exact, distances per the mode's
    # contract (a sample of rows; centroid-override rows are (c, 0))
    from conftest import assert_dist
    sys.path.insert(0, os.path.join(ROOT, "crypto-recommendation_amd"))
    import sharding as sh
    N, K = 120_000, 1024
    rows = sh.centroid_rows(N, K)
    Xall = oracle.synth(0x5EED, N, 128)
    sub = np.setdiff1d(np.random.default_rng(8).choice(N, 2000, replace=False), rows)
    oa, od = oracle.lloyd_assign(Xall[sub], Xall[rows].astype(np.float64), "euclidean", None)
    assert np.array_equal(cat("certified_assign0")[sub], oa)
    assert_dist(cat("certified_dist0")[sub], od, dist_mode)
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
    crow, crows = oracle.clusters_csr(one["certified_assign1"], K)
    want = oracle.cluster_top_n(Xall, np.zeros(N), crow, crows, Xall[qrows], np.zeros(96), one["recom_ucl1"], up,
                                np.concatenate(sets), 5)
    assert np.array_equal(one["recom_ucl1"], one["certified_assign1"][qrows])
    assert np.array_equal(one["recom1"], want)
    # hypercube: same coins, same engine state, same vertices
    for key in ("memo_f", "memo_h", "memo_bit", "memo_state"):
        for r in two:
            assert np.array_equal(r[key], one[key]), key
    assert np.array_equal(cat("vertex"), one["vertex"])
