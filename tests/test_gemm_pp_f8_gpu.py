"""The ping-pong projection GEMM on fp8 operands (csrc/gemm_pp.hip, F8 instantiations:
v_mfma_scale_f32_16x16x128_f8f6f4) against a plain PyTorch fp32 reference of the dequantised product:
plain store (e4m3 x e4m3 forward, e5m2 x e4m3 input gradient), M / N tails, strided operands, and the three
fused epilogues (RoPE, SwiGLU, SwiGLU backward) on the scaled accumulator."""
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
    form = G.set_mlp_coef(0)  # the gate / up saved form of the SwiGLU pair (the coefficient form: test_mlp_coef_gpu.py)
    torch.manual_seed(0)
    yield
    G.set_mlp_coef(form)
    ops.set_backend("auto")


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def maxrel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def q8(x, dt):
    """(fp8 tensor, dequantisation scale) with per-tensor current scaling."""
    fmax = 448.0 if dt == E4 else 57344.0
    s = fmax / x.abs().amax().clamp_min(1e-12) / 2
    return (x * s).to(dt), (1.0 / s).reshape(1).float()


def ref_mm(a8, sa, b8, sb):
    return (a8.float() @ b8.float().t()) * (sa * sb)


SHAPES = [(256, 256, 128), (512, 768, 256), (300, 264, 384), (1000, 520, 640), (4096, 3072, 1024),
          (2048, 2688, 1024), (8192, 1024, 5376), (64, 8, 128), (16384, 1024, 2688), (9000, 1000, 384),
          (2048, 32000, 1024), (2048, 1024, 32000)]


@pytest.mark.parametrize("adt", [E4, E5], ids=["e4m3", "e5m2"])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_pp_f8(M, N, K, adt):
    a8, sa = q8(torch.randn(M, K, device=DEV), adt)
    b8, sb = q8(torch.randn(N, K, device=DEV) * 0.05, E4)
    c = G.gemm_pp_f8(a8, b8, sa, sb)
    ref = ref_mm(a8, sa, b8, sb)
    assert c.dtype == torch.bfloat16
    assert rel(c, ref) < 5e-3
    assert maxrel(c, ref) < 1e-2


def test_gemm_pp_f8_matches_scaled_mm():
    M, N, K = 4096, 3072, 1024
    a8, sa = q8(torch.randn(M, K, device=DEV), E4)
    b8, sb = q8(torch.randn(N, K, device=DEV) * 0.05, E4)
    c = G.gemm_pp_f8(a8, b8, sa, sb)
    ref = torch._scaled_mm(a8, b8.t(), sa, sb, out_dtype=torch.bfloat16)
    assert rel(c, ref) < 5e-3


def test_gemm_pp_f8_strided():
    M, N, K = 600, 512, 256
    a_full, sa = q8(torch.randn(M, K + 128, device=DEV), E4)
    b_full, sb = q8(torch.randn(N + 8, K + 256, device=DEV) * 0.05, E4)
    a, b = a_full[:, 128:], b_full[8:, :K]
    out_full = torch.zeros(M, N + 96, device=DEV, dtype=torch.bfloat16)
    G.gemm_pp_f8(a, b, sa, sb, out_full[:, 32:32 + N])
    ref = ref_mm(a, sa, b, sb)
    assert rel(out_full[:, 32:32 + N], ref) < 5e-3
    assert out_full[:, :32].abs().max().item() == 0 and out_full[:, 32 + N:].abs().max().item() == 0


@pytest.mark.parametrize("hd", [64, 32])
def test_gemm_pp_rope_f8(hd):
    T, K = 256, 1024
    nq = 4 * hd * 3
    x8, sa = q8(torch.randn(2 * T, K, device=DEV), E4)
    w8, sb = q8(torch.randn(nq, K, device=DEV) * 0.05, E4)
    cos, sin = ops.rope_cache(T, hd, 10000.0, None, DEV)
    rc = 2 * nq // 3
    y = G.gemm_pp_rope_f8(x8, w8, sa, sb, cos, sin, T, hd, rc)
    ref = ref_mm(x8, sa, w8, sb)
    t = torch.arange(2 * T, device=DEV) % T
    q = ref[:, :rc].view(2 * T, -1, hd)
    c, s = cos[t].float()[:, None, :], sin[t].float()[:, None, :]
    rot = torch.cat([-q[..., hd // 2:], q[..., :hd // 2]], -1)
    ref[:, :rc] = (q * c + rot * s).reshape(2 * T, rc)
    assert rel(y, ref) < 5e-3


@pytest.mark.parametrize("M,F", [(1024, 672), (1000, 2688 // 4 + 8)])
def test_gemm_pp_swiglu_f8(M, F):
    K = 1024
    x8, sa = q8(torch.randn(M, K, device=DEV), E4)
    w8, sb = q8(torch.randn(2 * F, K, device=DEV) * 0.05, E4)
    gu, act = G.gemm_pp_swiglu_f8(x8, w8, sa, sb)
    ref = ref_mm(x8, sa, w8, sb)
    assert rel(gu, ref) < 5e-3
    g, u = gu[:, :F].float(), gu[:, F:].float()
    assert rel(act, torch.nn.functional.silu(g) * u) < 5e-3


@pytest.mark.parametrize("ddt", [E5, E4], ids=["e5m2", "e4m3"])
def test_gemm_pp_dswiglu_f8(ddt):
    M, F, K = 1024, 672, 1024
    gu = (torch.randn(M, 2 * F, device=DEV)).bfloat16()
    dy8, sa = q8(torch.randn(M, K, device=DEV), ddt)
    wdt8, sb = q8(torch.randn(F, K, device=DEV) * 0.05, E4)
    dgu = G.gemm_pp_dswiglu_f8(dy8, wdt8, sa, sb, gu)
    dact = ref_mm(dy8, sa, wdt8, sb)
    g, u = gu[:, :F].float(), gu[:, F:].float()
    sg = torch.sigmoid(g)
    ref = torch.cat([dact * u * sg * (1 + g * (1 - sg)), dact * g * sg], 1)
    assert rel(dgu, ref) < 5e-3


def test_gemm_pp_f8_deterministic():
    M, N, K = 4096, 1024, 2688 // 128 * 128
    a8, sa = q8(torch.randn(M, K, device=DEV), E5)
    b8, sb = q8(torch.randn(N, K, device=DEV) * 0.05, E4)
    c1 = G.gemm_pp_f8(a8, b8, sa, sb)
    c2 = G.gemm_pp_f8(a8, b8, sa, sb)
    assert torch.equal(c1, c2)


# ---------------------------------------------------------------- fp8 weight gradient (wgrad8_pp_kernel)
WG_SHAPES = [(256, 256, 128), (1024, 1024, 4096), (3072, 1024, 8192), (1024, 2688, 2048), (5376, 1024, 4096),
             (1000 // 16 * 16, 528, 1024), (2688, 1024, 384), (256, 32000 // 16 * 16, 256)]


@pytest.mark.parametrize("ddt", [E5, E4], ids=["e5m2", "e4m3"])
@pytest.mark.parametrize("M,N,K", WG_SHAPES)
def test_wgrad_f8(M, N, K, ddt):
    dy8, sdy = q8(torch.randn(K, M, device=DEV), ddt)
    x8, sx = q8(torch.randn(K, N, device=DEV), E4)
    gw0 = torch.randn(M, N, device=DEV)
    gw = gw0.clone()
    G.wgrad_f8(gw, dy8, x8, sdy, sx)
    ref = gw0 + (dy8.float().t() @ x8.float()) * (sdy * sx)
    assert rel(gw - gw0, ref - gw0) < 2e-3
    assert maxrel(gw - gw0, ref - gw0) < 1e-2


def test_wgrad_f8_strided_and_deterministic():
    K, M, N = 2048, 1024, 768
    dyf, sdy = q8(torch.randn(K, M + 64, device=DEV), E5)
    xf, sx = q8(torch.randn(K, N + 32, device=DEV), E4)
    dy8, x8 = dyf[:, 64:], xf[:, :N]
    out = []
    for _ in range(2):
        gw = torch.zeros(M, N, device=DEV)
        G.wgrad_f8(gw, dy8, x8, sdy, sx)
        out.append(gw)
    ref = (dy8.float().t() @ x8.float()) * (sdy * sx)
    assert rel(out[0], ref) < 2e-3
    assert torch.equal(out[0], out[1])


# ---------------------------------------------------------------- fp8 side outputs of the SwiGLU epilogues
def _cast(x, scale, dt):
    from nanodiloco_amd.ops import fp8
    return fp8.cast(x, scale, 0 if dt == E4 else 1)


@pytest.mark.parametrize("M,F", [(1024, 768), (1000, 640)])
def test_gemm_pp_swiglu_f8q_bitwise(M, F):
    """act8 from the epilogue == a separate cast of the plain form's bf16 act (bytes and amax)."""
    K = 1024
    x8, sa = q8(torch.randn(M, K, device=DEV), E4)
    w8, sb = q8(torch.randn(2 * F, K, device=DEV) * 0.05, E4)
    gu, act = G.gemm_pp_swiglu_f8(x8, w8, sa, sb)
    qs = torch.tensor([37.0], device=DEV)
    amax = torch.zeros(64, device=DEV)
    gu2, act8 = G.gemm_pp_swiglu_f8q(x8, w8, sa, sb, qs, amax)
    assert torch.equal(gu, gu2)
    assert torch.equal(act8.view(torch.uint8), _cast(act, qs, E4).view(torch.uint8))
    assert amax.max().item() == act.float().abs().max().item()


@pytest.mark.parametrize("ddt", [E5, E4], ids=["e5m2", "e4m3"])
def test_gemm_pp_dswiglu_f8q_bitwise(ddt):
    M, F, K = 1000, 640, 1024
    gu = torch.randn(M, 2 * F, device=DEV).bfloat16()
    dy8, sa = q8(torch.randn(M, K, device=DEV), ddt)
    wdt8, sb = q8(torch.randn(F, K, device=DEV) * 0.05, E4)
    dgu = G.gemm_pp_dswiglu_f8(dy8, wdt8, sa, sb, gu)
    qs = torch.tensor([900.0], device=DEV)
    amax = torch.zeros(64, device=DEV)
    dgu8 = G.gemm_pp_dswiglu_f8q(dy8, wdt8, sa, sb, gu, qs, amax)
    assert torch.equal(dgu8.view(torch.uint8), _cast(dgu, qs, E5).view(torch.uint8))
    assert amax.max().item() == dgu.float().abs().max().item()
