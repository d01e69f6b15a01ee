import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


def golden_meta():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        return json.load(f)


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def kpp_input(name):
    """Input rows of a k-means++ golden case (tests/golden/make_golden.py:kpp_data)."""
    import oracle
    m = golden_meta()[name]
    return oracle.synth(m["data_seed"], m["N"], m["d"])[np.arange(m["N"]) // m.get("dup", 1)]


def lloyd_input(name):
    """Input rows of a Lloyd golden case (tests/golden/make_golden.py:lloyd_data)."""
    import oracle
    m = golden_meta()[name]
    X = oracle.synth(m["data_seed"], m["N"], m["d"])
    z = m.get("zero_every", 0)
    if z:
        X[5::z] = 0.0
    return X


def case_rows(name):
    """Dataset rows of a golden case: stored fp64 rows (f64_* kinds) or the
    synthetic generator the case was made with (fp32)."""
    m = golden_meta()[name]
    g = golden(name)
    if "x64" in g.files:
        return g["x64"]
    kind = m["kind"]
    if kind in ("kmeanspp", "range"):
        return kpp_input(name)
    if kind == "lloyd":
        return lloyd_input(name)
    import oracle
    return oracle.synth(m["data_seed"], m["N"], m["d"])


def case_queries(name):
    """External query rows of an LSH / cube golden case."""
    m = golden_meta()[name]
    g = golden(name)
    if "q64" in g.files:
        return g["q64"]
    import oracle
    return oracle.synth(m["query_seed"], m["Q"], m["d"])


def cases(kind):
    return sorted(n for n, m in golden_meta().items() if m["kind"] == kind)


@pytest.fixture(scope="session")
def meta():
    return golden_meta()


# The distance contract is part of the C ABI (lshkm_ctx_set_dist_mode, the
# Conventions in include/lshkm.h): a context is in LSHKM_DIST_CERTIFIED mode by
# default (euclidean winner distances within 2^-20 relative -- the north star
# asks 1e-5 relative on float distances; cluster IDs and bucket IDs stay
# bit-exact) or, when set, LSHKM_DIST_EXACT (the reference-order fp64 chain, bit
# for bit). Tests taking `dist_mode` run both modes on their module's `ctx`; the
# rest run the shipped default. (The product library reads no environment; the
# LSHKM_DIST override exists only in the test build and is cleared for every
# test, so the ABI alone decides there too.)
DIST_TOL = 2.0 ** -20


@pytest.fixture(autouse=True)
def _no_dist_env(monkeypatch):
    monkeypatch.delenv("LSHKM_DIST", raising=False)


@pytest.fixture(params=["certified", "exact"])
def dist_mode(request):
    ctxs = [request.getfixturevalue("ctx")]
    if "sctx" in request.fixturenames:
        ctxs.append(request.getfixturevalue("sctx"))
    for c in ctxs:
        c.set_dist_mode(request.param)
    yield request.param
    for c in ctxs:
        c.set_dist_mode("certified")


@pytest.fixture(scope="session")
def sw():
    """The test build's binding (amd.switched()): forced kernel paths."""
    import amd
    return amd.switched()


@pytest.fixture(scope="module")
def sctx(sw):
    """A context of the test build (its handles are its own)."""
    import torch
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return sw.Context(0)


def assert_dist(got, want, mode, both_certified=False):
    """exact: bit for bit; certified: within DIST_TOL relative where the
    reference's distance is finite and non-zero, bit for bit elsewhere (0, inf,
    NaN). both_certified: `want` is itself a certified value (2 * DIST_TOL)."""
    got = np.ascontiguousarray(got, np.float64)
    want = np.ascontiguousarray(want, np.float64)
    assert got.shape == want.shape
    if mode == "exact":
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), np.nonzero(got != want)[0][:10]
        return
    assert mode in ("certified", "default"), mode
    fin = np.isfinite(want) & (want != 0.0)
    assert np.array_equal(got[~fin].view(np.uint64), want[~fin].view(np.uint64))
    rel = np.abs(got[fin] - want[fin]) / np.abs(want[fin])
    tol = DIST_TOL * (2.0 if both_certified else 1.0)
    assert rel.max(initial=0.0) <= tol, rel.max(initial=0.0)


