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
