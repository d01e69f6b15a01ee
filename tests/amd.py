"""Import helper for the product package (its directory name has a hyphen)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "crypto-recommendation_amd")


def load():
    spec = importlib.util.spec_from_file_location("lshkm_amd", os.path.join(PKG, "lshkm.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


lshkm = load()
