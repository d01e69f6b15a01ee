"""Import helper for the product package (its directory name has a hyphen)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "crypto-recommendation_amd")


def load(name="lshkm_amd", lib_path=None):
    spec = importlib.util.spec_from_file_location(name, os.path.join(PKG, "lshkm.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    if lib_path:
        mod.LIB_PATH = lib_path
    else:
        sys.modules.setdefault("lshkm", mod)     # cluster.py's `import lshkm` gets this same module
    return mod


lshkm = load()
_switched = None


def switched():
    """The same binding over the test build liblshkm_test.so: the product's
    sources with the A/B path switches compiled in (csrc/common.h test_switch,
    `make test`). Tests that force one kernel path against another run the
    forced path here and compare it with the product library (liblshkm.so,
    which reads no environment)."""
    global _switched
    if _switched is None:
        path = os.path.join(PKG, "liblshkm_test.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not built: run __graft_entry__.build()")
        _switched = load("lshkm_amd_switched", path)
    return _switched
