"""The coefficient form of the fused SwiGLU pair (csrc/gemm_pp.hip, FORM 1 of pp_epilogue; ops.gemm.set_mlp_coef):
the gate|up GEMM keeps A = d act / d gate and B = d act / d up instead of gate / up, the down-dgrad epilogue
multiplies.  Checked against the gate / up form (FORM 0) and plain fp32 PyTorch math, bf16 and fp8 (incl. the
fp8-output Q forms), and at the model level (ops.linear.MLPFn against the unfused chain)."""
import pytest
import torch

from nanodiloco_amd import ops
from nanodiloco_amd.ops import gemm as G

pytestmark = pytest.mark.gpu
DEV = "cuda"
E4, E5 = torch.float8_e4m3fn, torch.float8_e5m2


@pytest.fixture(autouse=True)
def _hip(hip_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.set_backend("hip")
    G.set_gemm_backend("hip")
    old = G.mlp_coef()
    torch.manual_seed(0)
    yield
    G.set_mlp_coef(old)
    ops.set_backend("auto")


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def coef_ref(gu):
    """[A | B] in fp32 from a gate / up form gu (the rounded gate / up the epilogue computes act from)."""
    F = gu.shape[1] // 2
    g, u = gu[:, :F].float(), gu[:, F:].float()
    s = torch.sigmoid(g)
    return torch.cat([u * s * (1 + g * (1 - s)), g * s], 1)


@pytest.mark.parametrize("M,F,K", [(1024, 672, 1024), (300, 136, 128), (4096, 2688, 1024), (2048, 5632, 2048)])
def test_coef_form_bf16_forward_and_backward(M, F, K):
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(2 * F, K, device=DEV) * 0.05).bfloat16()
    dy = torch.randn(M, 512, device=DEV).bfloat16()
    wdt = (torch.randn(F, 512, device=DEV) * 0.05).bfloat16()
    G.set_mlp_coef(0)
    gu, act0 = G.gemm_pp_swiglu(x, w)
    dgu0 = G.gemm_pp_dswiglu(dy, wdt, gu)
    G.set_mlp_coef(1)
    cf, act1 = G.gemm_pp_swiglu(x, w)
    assert torch.equal(act1, act0)  # act is computed exactly as in the gate / up form
    assert rel(cf, coef_ref(gu)) < 5e-3
    dgu1 = G.gemm_pp_dswiglu(dy, wdt, cf)
    dact = dy.float() @ wdt.float().t()
    ref = torch.cat([dact, dact], 1) * coef_ref(gu)
    assert rel(dgu1, ref) < 6e-3
    assert rel(dgu1, dgu0) < 8e-3


def _q8(x, dt):
    """(fp8 tensor, dequantisation scale), per-tensor current scaling (as tests/test_gemm_pp_f8_gpu.py)."""
    fmax = 448.0 if dt == E4 else 57344.0
    s = fmax / x.abs().amax().clamp_min(1e-12) / 2
    return (x * s).to(dt), (1.0 / s).reshape(1).float()


@pytest.mark.parametrize("ddt", [E5, E4], ids=["e5m2", "e4m3"])
def test_coef_form_fp8_forward_and_backward(ddt):
    M, F, K = 1024, 672, 1024
    x8, sa = _q8(torch.randn(M, K, device=DEV), E4)
    w8, sb = _q8(torch.randn(2 * F, K, device=DEV) * 0.05, E4)
    dy8, sd = _q8(torch.randn(M, K, device=DEV), ddt)
    wdt8, sw = _q8(torch.randn(F, K, device=DEV) * 0.05, E4)
    G.set_mlp_coef(0)
    gu, act0 = G.gemm_pp_swiglu_f8(x8, w8, sa, sb)
    dgu0 = G.gemm_pp_dswiglu_f8(dy8, wdt8, sd, sw, gu)
    qs, amax0 = torch.tensor([37.0], device=DEV), torch.zeros(64, device=DEV)
    _, act8_0 = G.gemm_pp_swiglu_f8q(x8, w8, sa, sb, qs, amax0)
    G.set_mlp_coef(1)
    cf, act1 = G.gemm_pp_swiglu_f8(x8, w8, sa, sb)
    assert torch.equal(act1, act0)
    assert rel(cf, coef_ref(gu)) < 5e-3
    amax1 = torch.zeros(64, device=DEV)
    cf2, act8_1 = G.gemm_pp_swiglu_f8q(x8, w8, sa, sb, qs, amax1)
    assert torch.equal(cf2, cf) and torch.equal(act8_1.view(torch.uint8), act8_0.view(torch.uint8))
    assert torch.equal(amax1, amax0)
    dgu1 = G.gemm_pp_dswiglu_f8(dy8, wdt8, sd, sw, cf)
    assert rel(dgu1, dgu0) < 8e-3
    dq, damax = torch.tensor([900.0], device=DEV), torch.zeros(64, device=DEV)
    dgu8 = G.gemm_pp_dswiglu_f8q(dy8, wdt8, sd, sw, cf, dq, damax)
    from nanodiloco_amd.ops import fp8
    assert torch.equal(dgu8.view(torch.uint8), fp8.cast(dgu1, dq, 1).view(torch.uint8))


def test_coef_form_fused_mlp_matches_unfused_chain():
    from tests.test_gemm_pp_gpu import _fused_vs_chain
    G.set_mlp_coef(1)
    f = _fused_vs_chain(True)
    u = _fused_vs_chain(False)
    for name, a, b in zip(["m", "o", "dy", "g_gu", "g_dn", "g_qkv"], f, u):
        assert rel(a, b) < 1e-2, name
