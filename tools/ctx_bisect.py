"""Diagnostic: run each test of tests/test_gpu_f64.py with its own Context,
destroying it explicitly after the test, printing a marker before and after,
to find which call sequence leaves the context unable to tear down."""
import inspect
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gc

import test_gpu_f64 as T
from amd import lshkm
from conftest import cases


class MP:
    def setenv(self, k, v):
        os.environ[k] = v


for name, fn in inspect.getmembers(T, inspect.isfunction):
    if not name.startswith("test_"):
        continue
    params = inspect.signature(fn).parameters
    runs = [dict()]
    if "name" in params:
        kind = {"test_f64_lsh_hash_build_query": "f64_lsh", "test_f64_cube": "f64_cube",
                "test_f64_lloyd_update_silhouette": "f64_lloyd", "test_f64_kmeans_pp": "f64_kmeanspp",
                "test_f64_range_assignment": "f64_range", "test_recommender_chain": "chain"}[name]
        runs = [dict(name=c) for c in cases(kind)]
    if "metric" in params:
        runs = [dict(r, metric=mt) for r in runs for mt in ("euclidean", "cosine")]
    if "path" in params:
        runs = [dict(r, path="auto", monkeypatch=MP()) for r in runs]
    for kw in runs:
        print("RUN", name, kw.get("name", ""), kw.get("metric", ""), flush=True)
        ctx = lshkm.Context(0)
        fn(ctx, **kw)
        os.environ.pop("LSHKM_ASSIGN_PATH", None)
        gc.collect()
        print("  close", flush=True)
        ctx.close()
        print("  closed", flush=True)
print("ALL OK", flush=True)
