"""Import helper for the product package (its directory name has a hyphen)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "crypto-recommendation_amd")


def load():
    spec = importlib.util.spec_from_file_location("lshkm_amd", os.path.join(PKG, "lshkm.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules.setdefault("lshkm", mod)     # cluster.py's `import lshkm` gets this same module
    return mod


lshkm = load()
