"""One-wave-per-SIMD projection GEMM (csrc/gemm_w128.hip) against a plain PyTorch fp32 reference:
single- and multi-tile persistent grids (the epilogue between tiles), M / N tails, strided operands
and output, determinism, a transposed-write check, and both tile orders."""
import pytest
import torch

from nanodiloco_amd import ops
from nanodiloco_amd.ops import gemm as G

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, params=[(4, 0), (1, 0), (3, 1), (4, 1)], ids=lambda p: f"gm{p[0]}-ovl{p[1]}")
def _hip(hip_lib, request):
    """Tile orders (grouped by 4 m-panels, row-major, a grouping with a short last group) x the two
    epilogue placements (between the tiles / inside each tile's last phase)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.set_backend("hip")
    gm, ovl = request.param
    old = G.set_w128(group_m=gm, ovl=ovl)
    torch.manual_seed(0)
    yield
    G.set_w128(group_m=old, ovl=0)
    ops.set_backend("auto")


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def maxrel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


SHAPES = [(256, 256, 64), (512, 768, 128), (300, 264, 192), (1000, 520, 640), (4096, 3072, 1024),
          (2048, 2688, 1024), (8192, 1024, 5376), (64, 8, 64), (256, 256, 128),
          (16384, 3072, 1024), (32768, 2688, 256), (9000, 1000, 320), (70000 // 8 * 8, 1032, 128),
          (2048, 32000, 1024), (2048, 1024, 32000), (2048, 2048, 2048), (1024, 2048, 11264)]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_w128(M, N, K):
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    c = G.gemm_w128(a, b)
    ref = a.float() @ b.float().t()
    assert rel(c, ref) < 5e-3
    assert maxrel(c, ref) < 1e-2


def test_gemm_w128_strided_operands_and_output():
    M, N, K = 600, 512, 256
    a_full = torch.randn(M, K + 64, device=DEV).bfloat16()
    b_full = (torch.randn(N + 8, K + 128, device=DEV) * 0.05).bfloat16()
    a, b = a_full[:, 64:], b_full[8:, :K]
    out_full = torch.zeros(M, N + 96, device=DEV, dtype=torch.bfloat16)
    out = out_full[:, 32:32 + N]
    G.gemm_w128(a, b, out)
    assert rel(out, a.float() @ b.float().t()) < 5e-3
    assert (out_full[:, :32] == 0).all() and (out_full[:, 32 + N:] == 0).all()


def test_gemm_w128_deterministic_and_plain_stores():
    a = torch.randn(4096, 1024, device=DEV).bfloat16()
    b = torch.randn(3072, 1024, device=DEV).bfloat16()
    c0 = G.gemm_w128(a, b)
    G.set_w128(nt=0)
    try:
        c1 = G.gemm_w128(a, b)
    finally:
        G.set_w128(nt=1)
    assert torch.equal(c0, G.gemm_w128(a, b)) and torch.equal(c0, c1)


def test_gemm_w128_identity_asymmetric():
    """A = I with an asymmetric B catches a transposed C write."""
    n = 512
    a = torch.eye(n, device=DEV).bfloat16()
    b = torch.randn(n, n, device=DEV).bfloat16()
    c = G.gemm_w128(a, b)
    assert torch.equal(c, b.t().contiguous())


@pytest.mark.parametrize("M,N,K", [s for s in SHAPES if s[2] >= 128])
def test_gemm_w128_vgpr_staged_b_bitwise(M, N, K):
    """The B operand staged through VGPRs (buffer_load + ds_write, round 6 A/B) writes the same LDS image as the
    LDS-DMA pieces: bitwise the same output (the variant runs with the epilogue inside the last phase; with the
    between-tiles placement of the fixture both calls take the DMA path)."""
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    c0 = G.gemm_w128(a, b)
    old = G.set_w128_vb(1)
    try:
        c1 = G.gemm_w128(a, b)
    finally:
        G.set_w128_vb(old)
    assert torch.equal(c0, c1)
    assert rel(c1, a.float() @ b.float().t()) < 5e-3
