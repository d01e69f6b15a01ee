"""The C++ drop-in (include/lshkm_compat.hpp).

CPU: the shim compiles against the reference's own headers (their
CustVector / CustHashtable / HashGenerator types) with g++ and plain C++14.
GPU: oracle/_ref/compat_check runs the reference's functions and the shim's
side by side through the reference's interface (hashtable buckets, queries,
filtered queries, hypercube probes, lloyds_assignment, k_means centers and
ownership) and must report no mismatch."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_LIB = "/root/reference/lib"
CHECK = os.path.join(ROOT, "oracle", "_ref", "compat_check")


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_LIB, "lsh_cube.hpp")), reason="reference headers absent")
def test_shim_compiles_against_reference_headers(tmp_path):
    src = tmp_path / "use_shim.cpp"
    src.write_text(
        '#include "utils.hpp"\n'
        '#include "lsh_cube.hpp"\n'
        '#include "clustering_phases/assignment.hpp"\n'
        '#include "clustering_phases/update.hpp"\n'
        '#include "clustering_phases/initialization.hpp"\n'
        '#include "lshkm_compat.hpp"\n'
        "template std::vector<CustHashtable<double>*> lshkm_compat::create_LSH_hashtables<double>(\n"
        "    std::vector<CustVector<double>>&, const std::string, int, int, int, double);\n"
        "template CustHashtable<double>* lshkm_compat::create_hypercube<double>(\n"
        "    std::vector<CustVector<double>>&, const std::string, int, double);\n"
        "template void lshkm_compat::lloyds_assignment<double>(std::vector<CustVector<double>>&,\n"
        "    std::vector<CustVector<double>*>&, std::string);\n"
        "template bool lshkm_compat::k_means<double>(std::vector<CustVector<double>>&,\n"
        "    std::vector<CustVector<double>*>&, std::string, double);\n"
        "template std::vector<CustVector<double>*> lshkm_compat::k_means_pp<double>(\n"
        "    std::vector<CustVector<double>>&, int, std::string);\n"
        "template std::vector<CustVector<double>*> lshkm_compat::rand_selection<double>(\n"
        "    std::vector<CustVector<double>>&, int);\n"
        "template std::vector<double> lshkm_compat::get_P_closest<double>(std::vector<CustVector<double>*>&,\n"
        "    CustVector<double>&, int);\n"
        "template std::vector<int> lshkm_compat::get_top_N_recom<double>(std::vector<CustVector<double>*>&,\n"
        "    CustVector<double>&, int, std::vector<double>);\n"
        "template std::vector<int> lshkm_compat::get_top_N_recom<double>(std::vector<CustVector<double>*>&,\n"
        "    CustVector<double>&, int);\n"
        "template class lshkm_compat::GpuLshGenerator<float>;\n"
        "template class lshkm_compat::GpuCubeGenerator<int>;\n")
    r = subprocess.run(["g++", "-std=c++14", "-fsyntax-only", "-Wall", "-Wno-unused-function", "-I", REF_LIB,
                        "-I", os.path.join(ROOT, "include"), str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    # and warning-free in the shim itself
    own = [ln for ln in r.stderr.splitlines() if re.search(r"lshkm_compat\.hpp:\d+:\d+: (warning|error)", ln)]
    assert not own, own


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["exact", "certified"])
@pytest.mark.parametrize("args", [("7", "2000", "128", "16"), ("11", "900", "17", "5"),
                                  ("13", "1500", "100", "12", "f64")])
def test_shim_matches_reference_functions(args, mode):
    # exact: the shim's default (LSHKM_DIST_EXACT) -- distances bit for bit, after
    # updates too (glibc's pow(x, 2), csrc/gpow2.h); certified:
    # lshkm_compat::set_distance_mode(LSHKM_DIST_CERTIFIED), euclidean distances
    # within 2^-20 relative. Everything else bit for bit in both.
    if not os.path.exists(CHECK):
        pytest.skip("oracle/_ref/compat_check not built (needs the reference sources at build time)")
    env = {k: v for k, v in os.environ.items() if k != "LSHKM_DIST"}   # the ABI mode alone decides
    r = subprocess.run([CHECK, *args, mode], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "compat ok" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
    # the comparison exercised something: non-empty filtered unions and probe
    # lists, and k_means replaced its centers at least once
    stats = dict(kv.split("=") for kv in r.stdout.split("compat ok")[1].split() if "=" in kv)
    assert stats["mode"] == mode
    if mode == "exact":
        assert int(stats["kmeans_euclidean_bitexact_iterations"]) == int(stats["kmeans_euclidean_iterations"]), stats
    for key in ("lsh_euclidean_filtered_rows", "lsh_cosine_filtered_rows", "cube_euclidean_probe_rows",
                "cube_cosine_probe_rows", "cluster_recom_users"):
        assert int(stats[key]) > 0, (key, stats)
    assert int(stats["kmeans_euclidean_iterations"]) >= 2 and int(stats["kmeans_cosine_iterations"]) >= 2, stats
    assert int(stats["recom_users"]) >= 30, stats
    # the per-user shim calls reused the cached clusters (main.cpp-shaped timing in the log)
    assert int(stats["cluster_recom_cache_hits"]) > 0, stats
    print("shim get_top_N_recom (3-argument, per user):", stats["cluster_recom_shim_us_per_user"], "us")
    assert int(stats["chain_users"]) >= 100, stats
