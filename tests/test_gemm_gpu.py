"""Own projection GEMMs (csrc/gemm.hip) against plain PyTorch fp32 references: plain NT product,
RoPE epilogue (q|k|v projection), SwiGLU epilogue (gate|up projection), SwiGLU-backward epilogue
(down-projection input gradient).  Shapes cover the Llama-150M / 1B projections, tails in M and N,
and GQA head layouts."""
import pytest
import torch

from nanodiloco_amd import ops
from nanodiloco_amd.ops import gemm as G
from nanodiloco_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, params=[(1, 0), (3, 4), (4, 0), (5, 3), (6, 4), (7, 0), (7, 4), (10, 4)], ids=lambda v: f"v{v[0]}g{v[1]}")
def _hip(hip_lib, request):
    """Every test runs on each schedule variant of the kernel (csrc/gemm.hip g_variant) and on a
    grouped tile order with a short last group (g_group_m = 3)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.set_backend("hip")
    G.set_gemm_backend("hip")
    old = G.set_gemm_variant(request.param[0])
    old_g = G.set_gemm_group_m(request.param[1])
    torch.manual_seed(0)
    yield
    G.set_gemm_variant(old)
    G.set_gemm_group_m(old_g)
    ops.set_backend("auto")


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


SHAPES = [(256, 256, 64), (1024, 768, 512), (777, 1000, 320), (300, 260, 128), (4096, 3072, 1024),
          (2048, 1024, 2688), (1024, 5376, 1024), (512, 32000, 1024), (64, 4, 64),
          (16384, 3072, 1024), (9000, 2056, 512)]  # the last two: several tiles per persistent workgroup


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_nt(M, N, K):
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    c = G.gemm_nt(a, b)
    assert rel(c, a.float() @ b.float().t()) < 5e-3


def test_gemm_nt_strided_operands_and_output():
    """Row-strided views (the fused q|k|v weight slice, a row block of a wider output)."""
    M, N, K = 600, 512, 256
    a_full = torch.randn(M, K + 64, device=DEV).bfloat16()
    b_full = (torch.randn(N + 8, K + 128, device=DEV) * 0.05).bfloat16()
    a, b = a_full[:, 64:], b_full[8:, :K]
    out_full = torch.zeros(M, N + 96, device=DEV, dtype=torch.bfloat16)
    out = out_full[:, 32:32 + N]
    G.gemm_nt(a, b, out)
    assert rel(out, a.float() @ b.float().t()) < 5e-3
    assert (out_full[:, :32] == 0).all() and (out_full[:, 32 + N:] == 0).all()


def test_gemm_nt_deterministic():
    a = torch.randn(2048, 1024, device=DEV).bfloat16()
    b = torch.randn(3072, 1024, device=DEV).bfloat16()
    assert torch.equal(G.gemm_nt(a, b), G.gemm_nt(a, b))


@pytest.mark.parametrize("B,T,nh,nkv,hd", [(2, 512, 16, 16, 64), (1, 1024, 8, 2, 64), (3, 128, 4, 4, 32),
                                           (2, 256, 8, 2, 32)])
def test_gemm_nt_rope(B, T, nh, nkv, hd):
    K = 256
    N = (nh + 2 * nkv) * hd
    x = torch.randn(B * T, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    cos, sin = ops.rope_cache(T, hd, 10000.0, None, DEV)
    out = G.gemm_nt_rope(x, w, cos, sin, T, hd, (nh + nkv) * hd)
    raw = x.float() @ w.float().t()
    q = raw[:, :nh * hd].view(B, T, nh, hd).transpose(1, 2)
    k = raw[:, nh * hd:(nh + nkv) * hd].view(B, T, nkv, hd).transpose(1, 2)
    q = ref.apply_rope(q, cos, sin).transpose(1, 2).reshape(B * T, nh * hd)
    k = ref.apply_rope(k, cos, sin).transpose(1, 2).reshape(B * T, nkv * hd)
    expect = torch.cat([q, k, raw[:, (nh + nkv) * hd:]], dim=1)
    assert rel(out, expect) < 5e-3
    # v columns are the plain product, bit for bit the plain kernel
    assert torch.equal(out[:, (nh + nkv) * hd:], G.gemm_nt(x, w)[:, (nh + nkv) * hd:])


@pytest.mark.parametrize("M,F,K", [(1024, 2688, 1024), (777, 300, 128), (256, 5632, 2048), (300, 128, 64)])
def test_gemm_nt_swiglu(M, F, K):
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(2 * F, K, device=DEV) * 0.05).bfloat16()
    gu, act = G.gemm_nt_swiglu(x, w)
    ref_gu = x.float() @ w.float().t()
    assert rel(gu, ref_gu) < 5e-3
    # act is computed from the rounded gate/up it stores (what the backward sees)
    g, u = gu[:, :F].float(), gu[:, F:].float()
    assert rel(act, torch.nn.functional.silu(g) * u) < 5e-3
    assert rel(act, ref.swiglu(ref_gu)) < 1e-2


@pytest.mark.parametrize("M,F,K", [(1024, 2688, 1024), (777, 300, 128), (256, 5632, 2048)])
def test_gemm_nt_dswiglu(M, F, K):
    dy = torch.randn(M, K, device=DEV).bfloat16()
    wt = (torch.randn(F, K, device=DEV) * 0.05).bfloat16()  # W_down^T [F, d]
    gu = torch.randn(M, 2 * F, device=DEV).bfloat16()
    dgu = G.gemm_nt_dswiglu(dy, wt, gu)
    gr = gu.float().requires_grad_(True)
    act = ref.swiglu(gr)
    (expect,) = torch.autograd.grad(act, gr, dy.float() @ wt.float().t())
    assert rel(dgu, expect) < 1e-2


def test_nt_supported_rejects_unaligned():
    a = torch.randn(64, 96, device=DEV).bfloat16()  # K % 64 != 0
    b = torch.randn(64, 96, device=DEV).bfloat16()
    assert not G.nt_supported(a, b)
    a = torch.randn(64, 128, device=DEV).bfloat16()
    b = torch.randn(64, 128, device=DEV).bfloat16()
    assert G.nt_supported(a, b)
