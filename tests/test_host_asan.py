"""Host sanitizer run: liblshkm's host parsers (csrc/io.cpp — the
CSV vector reader, cluster.conf / file_to_args, ArgParser) compiled with
-fsanitize=address,undefined on the host side only (hipcc -Xarch_host; no GPU
code is instrumented) and run over the committed format fixtures and generated
malformed inputs (tests/host_asan.cpp). CPU only."""
import glob
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="needs hipcc")
def test_host_parsers_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_asan")
    cmd = [HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O1", "-g", "-std=c++17",
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "crypto-recommendation_amd", "csrc"),
           os.path.join(HERE, "host_asan.cpp"), "-o", exe, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    fixtures = sorted(glob.glob(os.path.join(HERE, "golden", "io", "*")))
    assert fixtures
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    work = tmp_path / "work"
    work.mkdir()
    r = subprocess.run([exe, str(work)] + fixtures, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "host_asan ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    shutil.rmtree(work, ignore_errors=True)
