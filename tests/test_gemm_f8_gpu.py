"""Own fp8 projection GEMM (csrc/gemm.hip gemm4_f8_kernel, v_mfma_scale_f32_32x32x64_f8f6f4) against
an fp32 PyTorch reference of the dequantised operands and against ``torch._scaled_mm`` (the hipBLASLt
path it replaces in ops/fp8.py): forward e4m3 x e4m3 and input-gradient e5m2 x e4m3, tails in M and
N, strided operands, and grids with several tiles per persistent workgroup."""
import pytest
import torch

from nanodiloco_amd import ops
from nanodiloco_amd.ops import gemm as G

pytestmark = pytest.mark.gpu
DEV = "cuda"
E4, E5 = torch.float8_e4m3fn, torch.float8_e5m2


@pytest.fixture(autouse=True, params=[-1, 0, 1, 2, 3], ids=lambda v: f"ldm{v}")
def _hip(hip_lib, request):
    """Every loader variant of the kernel (csrc/gemm.hip g_f8_variant: DMA burst, DMA interleaved,
    VGPR staging)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    old = G.set_gemm_f8_variant(request.param)
    torch.manual_seed(0)
    yield
    G.set_gemm_f8_variant(old)


def q8(x, dt):
    fmax = torch.finfo(dt).max
    s = fmax / x.abs().amax().clamp_min(1e-12)
    return (x * s).clamp(-fmax, fmax).to(dt), (1.0 / s).reshape(1).float()


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("fa", [E4, E5], ids=["e4m3", "e5m2"])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (777, 1000, 384), (300, 264, 128), (4096, 3072, 1024),
                                   (16384, 3072, 1024), (65536, 1024, 2688), (8192, 5376, 1024)])
def test_gemm_nt_f8(M, N, K, fa):
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(N, K, device=DEV) * 0.05
    a8, sa = q8(a, fa)
    b8, sb = q8(b, E4)
    c = G.gemm_nt_f8(a8, b8, sa, sb)
    expect = (a8.float() * sa) @ (b8.float() * sb).t()
    assert c.dtype == torch.bfloat16 and c.shape == (M, N)
    assert rel(c, expect) < 4e-3
    if N % 16 == 0:  # hipBLASLt's fp8 path needs 16-multiples
        lib = torch._scaled_mm(a8, b8.t(), sa, sb, out_dtype=torch.bfloat16)
        assert rel(c, lib) < 4e-3


def test_gemm_nt_f8_strided_and_deterministic():
    M, N, K = 1000, 512, 256
    a_full, sa = q8(torch.randn(M, K + 128, device=DEV), E4)
    b_full, sb = q8(torch.randn(N + 8, K + 256, device=DEV), E4)
    a, b = a_full[:, 128:], b_full[8:, :K]
    out_full = torch.zeros(M, N + 64, device=DEV, dtype=torch.bfloat16)
    out = out_full[:, 32:32 + N]
    G.gemm_nt_f8(a, b, sa, sb, out)
    expect = (a.float() * sa) @ (b.float() * sb).t()
    assert rel(out, expect) < 4e-3
    assert (out_full[:, :32] == 0).all() and (out_full[:, 32 + N:] == 0).all()
    assert torch.equal(G.gemm_nt_f8(a, b, sa, sb), G.gemm_nt_f8(a, b, sa, sb))


def test_f8_nt_supported():
    a8 = torch.zeros(64, 192, device=DEV, dtype=E4)  # K % 128 != 0
    assert not G.f8_nt_supported(a8, a8)
    a8 = torch.zeros(64, 256, device=DEV, dtype=E4)
    assert G.f8_nt_supported(a8, a8)
