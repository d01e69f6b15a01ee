"""Config C1 end to end (BASELINE.json configs[0], main.cpp:81-111): a 1k x 16
CSV read through cluster.conf, k-means++ (cosine), Lloyd + k-means until
convergence, on the MI355X path — against the reference's own run of the same
block on the same file (tests/golden c1_* fixtures)."""
import os
import sys

import numpy as np
import pytest

from amd import PKG, lshkm
from conftest import GOLDEN, cases, golden, golden_meta

sys.path.insert(0, PKG)
import cluster  # noqa: E402

META = golden_meta()
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return lshkm.Context(0)


@pytest.mark.parametrize("name", cases("c1"))
def test_c1_matches_reference(ctx, name, tmp_path):
    m, g = META[name], golden(name)
    conf = tmp_path / "cluster.conf"
    conf.write_text(f"proj_2_input {os.path.join(GOLDEN, m['file'])}\nproj_2_csv_delimiter ,\n"
                    f"proj_2_number_of_clusters {m['K']}\nnumber_of_clusters 30\n"
                    f"max_algo_iterations {m['iters']}\nmin_dist_kmeans {m['min_dist']!r}\n")
    res = cluster.run_proj2(ctx, str(conf), m["seed"])
    assert res["ids"] == [str(i) for i in range(m["N"])]
    assert np.array_equal(res["rows"], g["kpp_rows"])
    it = int(g["iters"][0])
    assert res["iters"] == it and res["cont"] == bool(g["cont"][0])
    assert np.array_equal(res["assign"], g[f"assign{it - 1}"])
    # the last iteration's centroids are k-means means (general fp64): the
    # reference's distances bit for bit (glibc's pow(x, 2), csrc/gpow2.h)
    want = g[f"dist{it - 1}"]
    assert np.array_equal(res["dist"].view(np.uint64), want.view(np.uint64))
    # centers after the last k_means (replaced iff it continued): bit-exact sums
    assert np.array_equal(res["centers"].view(np.uint64), g[f"centers{it}"].view(np.uint64))
