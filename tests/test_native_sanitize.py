"""Host-code sanitizer run: the native token loader built with ASan + UBSan and
driven by a C++ harness across epochs, ring depths and seek/resume."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "nanodiloco_amd", "csrc", "runtime")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_token_loader_asan_ubsan(tmp_path):
    exe = tmp_path / "t"
    r = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                        "-pthread", os.path.join(RT, "token_loader.cpp"), os.path.join(RT, "test_token_loader.cpp"),
                        "-o", str(exe)], capture_output=True, text=True)
    if r.returncode != 0 and "asan" in r.stderr.lower():
        pytest.skip("ASan runtime unavailable")
    assert r.returncode == 0, r.stderr
    data = tmp_path / "d.bin"
    np.arange(50 * 16, dtype=np.uint16).tofile(data)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe), str(data)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
