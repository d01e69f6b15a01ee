"""CPU-side checks of the product's host code (no GPU needed):
the C-ABI library loads and exports every symbol include/lshkm.h declares,
the host parameter generation reproduces the reference's RNG draws bit for
bit, the soft-x87 emulation used by the kernels' exact paths agrees with
real x87 long double, and the restatement of glibc's pow(x, 2) (csrc/gpow2.h)
agrees with this process's pow."""
import os
import subprocess

import numpy as np
import pytest

import oracle
from amd import PKG, ROOT, lshkm
from conftest import cases, golden, golden_meta

META = golden_meta()


def test_library_exports_declared_symbols():
    L = lshkm.lib()
    declared = lshkm.declared_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    assert lshkm.lib().lshkm_version().decode().startswith("lshkm-gfx950")


def test_binding_declares_every_abi_signature():
    # ctypes without argtypes passes ints as 32-bit: every ABI entry point needs
    # an explicit signature in lshkm.lib()'s table
    L = lshkm.lib()
    untyped = [s for s in lshkm.declared_symbols() if getattr(L, s).argtypes is None]
    assert not untyped, untyped


def test_library_is_gfx950_code_object():
    with open(os.path.join(PKG, "liblshkm.so"), "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


@pytest.mark.parametrize("name", cases("lsh"))
def test_params_lsh_match_reference(name):
    m, g = META[name], golden(name)
    if m["metric"] == "euclidean":
        V, t, r, st = lshkm.params_lsh_euclidean(m["seed"], m["L"], m["k"], m["d"], m["w"])
        assert np.array_equal(V, g["V"]) and np.array_equal(t, g["t"]) and np.array_equal(r, g["r"])
        assert st == oracle.gen_lsh_euclid(m["seed"], m["L"], m["k"], m["d"], np.float32(m["w"]))[3]
    else:
        R, st = lshkm.params_lsh_cosine(m["seed"], m["L"], m["k"], m["d"])
        assert np.array_equal(R.view(np.uint64), g["R"].view(np.uint64))
        assert st == oracle.gen_lsh_cosine(m["seed"], m["L"], m["k"], m["d"])[1]


@pytest.mark.parametrize("name", cases("cube"))
def test_params_cube_match_reference(name):
    m, g = META[name], golden(name)
    if m["metric"] == "euclidean":
        V, t, st = lshkm.params_cube_euclidean(m["seed"], m["k"], m["d"], m["w"])
        assert np.array_equal(V, g["V"]) and np.array_equal(t, g["t"])
        assert st == oracle.gen_cube_euclid(m["seed"], m["k"], m["d"], np.float32(m["w"]))[2]
    else:
        R, st = lshkm.params_cube_cosine(m["seed"], m["k"], m["d"])
        assert np.array_equal(R.view(np.uint64), g["R"].view(np.uint64))


@pytest.mark.parametrize("name", cases("kmeanspp"))
def test_rand_selection_matches_reference(name):
    # host-only entry point (lshkm_rand_selection): no GPU needed
    m = META[name]
    assert np.array_equal(lshkm.rand_selection_rows(m["N"], m["K"], m["seed"]), golden(name)["rand_rows"])


def test_rand_selection_rejects_k_above_n():
    with pytest.raises(lshkm.LshkmError):
        lshkm.rand_selection_rows(3, 4, 1)      # the reference would loop forever


def test_params_bad_arguments_fail_loudly():
    with pytest.raises(lshkm.LshkmError):
        lshkm.params_lsh_euclidean(1, 0, 4, 128, 0.4)


def test_softx87_matches_long_double(tmp_path):
    exe = tmp_path / "softx87_check"
    subprocess.run(["g++", "-O1", "-std=c++14", "-o", str(exe), os.path.join(ROOT, "tests", "softx87_check.cpp")],
                   check=True)
    out = subprocess.run([str(exe), "100000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad=0" in out.stdout


def test_kmseg_matches_chain(tmp_path):
    # the binade-segment evaluation of the fp64 chain (csrc/kmseg.h) vs the plain chain
    exe = tmp_path / "kmseg_check"
    subprocess.run(["g++", "-O1", "-std=c++14", "-o", str(exe), os.path.join(ROOT, "tests", "kmseg_check.cpp")],
                   check=True)
    out = subprocess.run([str(exe), "30"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad=0" in out.stdout


def test_pow2_restatement_matches_glibc(tmp_path):
    # csrc/gpow2.h (glibc 2.35 __pow_fma, operation for operation) vs the real
    # pow on 7 x 4M inputs: any bit pattern, [0.5, 4), exact ties, the special
    # ranges, random exponents, squares within 2^-8 ulp of a midpoint (a fifth
    # of which differ from x*x) and exact squares of every exponent
    exe = tmp_path / "pow2_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fopenmp", "-o", str(exe),
                    os.path.join(ROOT, "tests", "pow2_check.cpp"), "-lm"], check=True)
    out = subprocess.run([str(exe), "4"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "total mismatches 0" in out.stdout
    differ = int(out.stdout.split("pow != x*x on ")[-1].split()[0])
    assert differ > 100_000, out.stdout            # the inputs do tell pow from x*x


def test_pow_selfcheck_in_library():
    # the library's own host-side check against the process's pow (lshkm_pow_selfcheck)
    bad, tested = lshkm.pow_selfcheck()
    assert bad == 0 and tested >= 6000, (bad, tested)


def test_release_library_reads_no_environment():
    # the product library takes no path switches from the environment: no getenv
    # import at all (the A/B switches live in liblshkm_test.so only)
    syms = subprocess.run(["nm", "-D", "--undefined-only", os.path.join(PKG, "liblshkm.so")], capture_output=True,
                          text=True, check=True).stdout
    assert " getenv" not in syms and "secure_getenv" not in syms, [l for l in syms.splitlines() if "getenv" in l]
    test_syms = subprocess.run(["nm", "-D", "--undefined-only", os.path.join(PKG, "liblshkm_test.so")],
                               capture_output=True, text=True, check=True).stdout
    assert " getenv" in test_syms


def test_no_gpu_means_loud_failure():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(Exception):
        lshkm.Context(0)


_CTX_PROBE = r"""
import ctypes, sys
L = ctypes.CDLL(sys.argv[1])
L.lshkm_last_error.restype = ctypes.c_char_p
h = ctypes.c_void_p()
rc = L.lshkm_ctx_create(0, ctypes.byref(h))
print(rc, L.lshkm_last_error().decode())
if rc == 0:
    L.lshkm_ctx_destroy(h)
"""


def _ctx_create_in_child(libname, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    out = subprocess.run([os.sys.executable, "-c", _CTX_PROBE, os.path.join(PKG, libname)], capture_output=True,
                         text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    rc, msg = out.stdout.strip().split(" ", 1) if " " in out.stdout.strip() else (out.stdout.strip(), "")
    return int(rc), msg


def test_ctx_create_enforces_pow_contract():
    # lshkm_ctx_create runs lshkm_pow_selfcheck once per process, before any
    # device work, and refuses on a host whose pow(x, 2) is not the one the
    # device restates (gpow2.h). The test build's LSHKM_POW_HOST=rn stands in
    # for such a host (a correctly rounded square): refused with
    # LSHKM_ERR_UNSUPPORTED and the mismatch count, GPU or not.
    rc, msg = _ctx_create_in_child("liblshkm_test.so", {"LSHKM_POW_HOST": "rn"})
    assert rc == -4 and "pow(x, 2) differs" in msg, (rc, msg)
    bad = int(msg.split(" on ")[1].split(" of ")[0])
    assert bad > 100, msg                          # the self-check's inputs tell pow from x*x
    # this image's libm: the contract holds; the context then fails only for want
    # of a GPU here (or succeeds on the GPU box)
    for lib in ("liblshkm.so", "liblshkm_test.so"):
        rc, msg = _ctx_create_in_child(lib, {"LSHKM_POW_HOST": "rn"} if lib == "liblshkm.so" else {})
        assert "pow" not in msg, (lib, rc, msg)    # the product library reads no switch
