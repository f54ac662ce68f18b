"""The product kernel library contains no wrong-result timing ablation (verdict r4 weak #6): the ablation
instantiations exist only in the -DND_ABLATION build (csrc/build.py --ablation -> _lib/alt/), the correct
A/B switches are read once when the library loads, and the ablation environment variables / setters
cannot select anything else (CPU: the library loads without a GPU; no kernel is launched)."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "nanodiloco_amd", "_lib", "libnd_kernels.so")


def _symbols():
    if not os.path.exists(LIB) or shutil.which("nm") is None:
        pytest.skip("kernel library not built / nm missing")
    out = subprocess.run(["nm", "-C", LIB], capture_output=True, text=True, check=True).stdout
    return [ln for ln in out.splitlines() if "_kernel<" in ln]


def _targs(line, name):
    m = re.search(re.escape(name) + r"<([^>]*)>", line)
    return [x.strip() for x in m.group(1).split(",")] if m else None


def test_default_library_has_no_ablation_instantiation():
    syms = _symbols()
    seen = {"attn_fwd_kernel": 0, "attn_bwd_dkdv_dma_kernel": 0, "gemm_pp_kernel": 0, "gemm_w128_kernel": 0,
            "wgrad_pp_kernel": 0}
    for ln in syms:
        for name in seen:
            t = _targs(ln, " " + name) or _targs(ln, name)
            if t is None or not re.search(r"\b" + name + "<", ln):
                continue
            seen[name] += 1
            if name == "attn_fwd_kernel" and len(t) >= 5:
                assert t[4] in ("0", "32"), ln  # ABL: 32 is the correct default variant
            elif name == "attn_bwd_dkdv_dma_kernel" and len(t) >= 6:
                assert t[5] == "0", ln
            elif name == "gemm_pp_kernel":
                assert t[2] in ("0", "32", "256", "288", "512", "1024", "2048", "2080"), ln  # 512 / 2048 / 2080: store policy
            elif name == "gemm_w128_kernel":
                assert t[3] == "0", ln
            elif name == "wgrad_pp_kernel" and len(t) >= 2:
                assert t[1] == "0", ln
    assert all(v > 0 for v in seen.values()), seen  # the parse found the kernels at all
    assert not any("wgrad_dma_kernel<true, true>" in ln for ln in syms)  # "nodma" diagnostic
    assert not any("nd_attn_ablation_build" in ln for ln in syms)


_PROBE = r'''
import ctypes, sys
lib = ctypes.CDLL(sys.argv[1])
# the ablation setters refuse every wrong-result variant in the product library
assert lib.nd_gemm_pp_set_variant(1) == -1 and lib.nd_gemm_pp_set_variant(128) == -1
assert lib.nd_gemm_pp_set_variant(0) == 0  # the environment's ND_GEMM_PP_VARIANT=1 was ignored at load
assert lib.nd_gemm_w128_set_ablation(1) == -1
assert not hasattr(lib, "nd_attn_ablation_build")
print("GATE_OK")
'''


def test_ablation_env_cannot_select_variants():
    if not os.path.exists(LIB):
        pytest.skip("kernel library not built")
    env = dict(os.environ, ND_ATTN_DKDV_ABL="1", ND_ATTN_ABL="4", ND_GEMM_PP_VARIANT="1", ND_WGRAD_VARIANT="a1",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-c", _PROBE, LIB], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "GATE_OK" in r.stdout, r.stdout + r.stderr
