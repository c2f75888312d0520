"""The host C/C++ under AddressSanitizer + UndefinedBehaviorSanitizer: the C ABI's host
code (cbf_amd/csrc/abi.cpp) and the C oracle (oracle/cbf_oracle.c), built with
-fsanitize=address,undefined and driven by tests/sanitize/driver.c on random and edge inputs.
CPU only; the HIP kernels are checked by the GPU parity suite (GPU sanitizers are not available on
the GPU pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None, reason="needs gcc/g++")
def test_host_code_under_asan_ubsan(tmp_path):
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
    inc = ["-I", os.path.join(ROOT, "include")]
    objs = []
    for src, comp, extra in ((os.path.join(ROOT, "oracle", "cbf_oracle.c"), "gcc", ["-ffp-contract=off"]),
                             (os.path.join(ROOT, "cbf_amd", "csrc", "abi.cpp"), "g++", ["-std=c++17"]),
                             (os.path.join(ROOT, "tests", "sanitize", "driver.c"), "gcc", [])):
        o = str(tmp_path / (os.path.basename(src) + ".o"))
        subprocess.run([comp, *san, *extra, *inc, "-c", src, "-o", o], check=True)
        objs.append(o)
    exe = str(tmp_path / "driver")
    subprocess.run(["g++", *san, *objs, "-o", exe, "-lm"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "sanitize driver ok" in r.stdout
