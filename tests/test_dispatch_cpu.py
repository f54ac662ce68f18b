"""CPU checks of the op-dispatch switches added in round 2: fp8 GEMM backend selection, the own
fp8 GEMM's shape gate, and the lm-head chunking rule (one chunk per 64k-token micro-batch)."""
import pytest
import torch

from nanodiloco_amd.ops import cross_entropy as ce
from nanodiloco_amd.ops import fp8
from nanodiloco_amd.ops import gemm as G


def test_fp8_gemm_backend_switch():
    old = fp8.fp8_gemm_backend()
    assert old == "pp"  # own fp8 ping-pong kernel + fused epilogues for every product (profiles/r4_fp8_pp.md)
    assert fp8.fp8_fused_epilogues()
    try:
        fp8.set_fp8_gemm("auto")
        assert fp8.fp8_fused_epilogues()
        fp8.set_fp8_gemm("hipblaslt")
        assert fp8.fp8_gemm_backend() == "hipblaslt"
        assert not fp8.fp8_fused_epilogues()  # the fused fp8 epilogues live in the pp kernel only
        for bad in ("cublas", "hip"):  # "hip" (the round-2 fp8 kernel) was removed in round 5
            with pytest.raises(ValueError):
                fp8.set_fp8_gemm(bad)
    finally:
        fp8.set_fp8_gemm(old)


def test_pp_f8_supported_gate_on_cpu():
    a = torch.zeros(256, 256, dtype=torch.float8_e4m3fn)
    assert not G.pp_f8_supported(a, a)  # CPU tensors never take the HIP kernel


def test_lm_head_chunk_rows():
    # 4 GiB budget: a whole 65,536-row micro-batch of a 32k vocabulary in bf16 is one chunk
    assert ce._chunk_rows(32000, 2) >= 65536
    assert ce._chunk_rows(32000, 2) % 256 == 0
    assert ce._chunk_rows(32000, 2, budget_bytes=1 << 30) == 16640  # (4 equal chunks of 16384 in the forward)
    assert ce._chunk_rows(10 ** 9, 4) == 256  # never below one 256-row block


def test_lm_head_ce_chunked_matches_unchunked():
    torch.manual_seed(0)
    n, d, V = 600, 32, 50
    y = torch.randn(n, d, requires_grad=True)
    w = torch.randn(V, d) * 0.1
    t = torch.randint(0, V, (n,))
    t[::7] = ce.IGNORE_INDEX
    gw1, gw2 = torch.zeros(V, d), torch.zeros(V, d)
    l1 = ce.lm_head_ce(y, w, gw1, t, chunk_rows=256)
    (g1,) = torch.autograd.grad(l1, y)
    l2 = ce.lm_head_ce(y, w, gw2, t)
    (g2,) = torch.autograd.grad(l2, y)
    assert torch.allclose(l1, l2, atol=1e-5)
    assert torch.allclose(g1, g2, atol=1e-6)
    assert torch.allclose(gw1, gw2, atol=1e-5)


def test_fp8_keep_fused_routing():
    """--fp8-keep-fused: which decoder projections stay fp8 (measured default: all of them,
    profiles/r3_fp8_keep_fused_ab.md)."""
    assert fp8.fp8_keep_fused() == {"rope": False, "mlp": False}
    want = {"none": {"qkv", "o", "gu", "down"}, "rope": {"o", "gu", "down"}, "mlp": {"qkv", "o"}, "both": {"o"}}
    try:
        for mode, kinds in want.items():
            fp8.set_fp8_keep_fused(mode)
            assert {k for k in ("qkv", "o", "gu", "down") if fp8.fp8_projection(k)} == kinds
        with pytest.raises(ValueError):
            fp8.set_fp8_keep_fused("all")
    finally:
        fp8.set_fp8_keep_fused("none")


def test_proj_gemm_modes():
    """Plain projection GEMM routing: hipBLASLt by default; 'short' / 'pp' select the own kernel
    (never on CPU tensors); unknown names are rejected."""
    import importlib

    L = importlib.import_module("nanodiloco_amd.ops.linear")  # (ops.linear is the re-exported function)

    assert L.proj_gemm() == "blas"
    a, b = torch.randn(64, 128), torch.randn(32, 128)
    try:
        for mode in ("blas", "short", "pp"):
            L.set_proj_gemm(mode)
            assert not L._pp_ok(a, b)  # CPU tensors always take torch.mm
            assert torch.allclose(L.mm_nt(a, b), a @ b.t())
        with pytest.raises(ValueError):
            L.set_proj_gemm("cublas")
    finally:
        L.set_proj_gemm("blas")


def test_fp8_auto_dispatch_rule():
    a = torch.zeros(4096, 1024, dtype=torch.float8_e4m3fn)
    assert fp8._own_plain(a, torch.zeros(1024, 1024, dtype=torch.float8_e4m3fn))  # K = 1024: own kernel
    assert fp8._own_plain(a, torch.zeros(2688, 1024, dtype=torch.float8_e4m3fn))
    long_k = torch.zeros(4096, 5376, dtype=torch.float8_e5m2)
    assert not fp8._own_plain(long_k, torch.zeros(1024, 5376, dtype=torch.float8_e4m3fn))  # hipBLASLt
