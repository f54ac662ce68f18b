"""Ping-pong projection GEMM (csrc/gemm_pp.hip) against plain PyTorch fp32 references: plain NT
product (single- and multi-tile persistent grids, M / N tails, strided operands and output), the
RoPE / SwiGLU / SwiGLU-backward epilogues, and the model-level fused ops built on them
(ops.linear.LinearRopeFn, MLPFn) against the unfused op chains, forward and backward."""
import pytest
import torch

from nanodiloco_amd import ops
from nanodiloco_amd.ops import gemm as G

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, params=[4, 1, 3], ids=lambda g: f"gm{g}")
def _hip(hip_lib, request):
    """Every test runs with the default grouped tile order (4 m-panels), the plain row-major order
    and a grouping that leaves a short last group."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.set_backend("hip")
    G.set_gemm_backend("hip")
    old = G.set_pp_group_m(request.param)
    form = G.set_mlp_coef(0)  # these tests pin the gate / up saved form (the coefficient form: test_mlp_coef_gpu.py)
    torch.manual_seed(0)
    yield
    G.set_mlp_coef(form)
    G.set_pp_group_m(old)
    ops.set_backend("auto")


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def maxrel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


SHAPES = [(256, 256, 64), (512, 768, 128), (300, 264, 192), (1000, 520, 640), (4096, 3072, 1024),
          (2048, 2688, 1024), (8192, 1024, 5376), (64, 8, 64),
          # several tiles per persistent workgroup (the epilogue inside the next tile's first phase)
          (16384, 3072, 1024), (32768, 2688, 256), (9000, 1000, 320), (70000 // 8 * 8, 1032, 128),
          # Llama-150M lm head logits / dgrad, and the Llama-1B plain projections (o / down fwd, q|k|v,
          # o and gate|up dgrad, lm head) at reduced M
          (2048, 32000, 1024), (2048, 1024, 32000), (2048, 2048, 2048), (2048, 2048, 5632), (2048, 2048, 2560),
          (1024, 2048, 11264), (1024, 32000, 2048), (1024, 2048, 32000)]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_pp(M, N, K):
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    c = G.gemm_pp(a, b)
    ref = a.float() @ b.float().t()
    assert rel(c, ref) < 5e-3
    assert maxrel(c, ref) < 1e-2


def test_gemm_pp_strided_operands_and_output():
    """Row-strided views (the fused q|k|v weight slice, a column block of a wider output)."""
    M, N, K = 600, 512, 256
    a_full = torch.randn(M, K + 64, device=DEV).bfloat16()
    b_full = (torch.randn(N + 8, K + 128, device=DEV) * 0.05).bfloat16()
    a, b = a_full[:, 64:], b_full[8:, :K]
    out_full = torch.zeros(M, N + 96, device=DEV, dtype=torch.bfloat16)
    out = out_full[:, 32:32 + N]
    G.gemm_pp(a, b, out)
    assert rel(out, a.float() @ b.float().t()) < 5e-3
    assert (out_full[:, :32] == 0).all() and (out_full[:, 32 + N:] == 0).all()


def test_gemm_pp_deterministic():
    a = torch.randn(4096, 1024, device=DEV).bfloat16()
    b = torch.randn(3072, 1024, device=DEV).bfloat16()
    assert torch.equal(G.gemm_pp(a, b), G.gemm_pp(a, b))


def test_gemm_pp_identity_asymmetric():
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    n = 512
    a = torch.eye(n, device=DEV).bfloat16()
    b = (torch.arange(n * n, device=DEV, dtype=torch.float32).view(n, n) % 251 - 125).bfloat16()
    c = G.gemm_pp(a, b)  # = I . b^T = b^T
    assert torch.equal(c, b.t().contiguous())


@pytest.mark.parametrize("B,T,nh,nkv,hd", [(2, 512, 16, 16, 64), (1, 1024, 8, 2, 64), (3, 128, 4, 4, 32),
                                           (2, 256, 8, 2, 32), (8, 1024, 16, 16, 64),
                                           (2, 1024, 32, 4, 64)])  # Llama-1B q|k|v (N = 2560)
def test_gemm_pp_rope(B, T, nh, nkv, hd):
    K = 256
    N = (nh + 2 * nkv) * hd
    x = torch.randn(B * T, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    cos, sin = ops.rope_cache(T, hd, 10000.0, None, DEV)
    rc = (nh + nkv) * hd
    out = G.gemm_pp_rope(x, w, cos, sin, T, hd, rc)
    ref = x.float() @ w.float().t()
    t = torch.arange(B * T, device=DEV) % T
    q = ref[:, :rc].view(B * T, -1, hd)
    c, s = cos[t].float()[:, None, :], sin[t].float()[:, None, :]
    rot = torch.cat([-q[..., hd // 2:], q[..., :hd // 2]], -1)
    ref[:, :rc] = (q * c + rot * s).reshape(B * T, rc)
    assert rel(out, ref) < 5e-3
    assert maxrel(out, ref) < 1e-2


@pytest.mark.parametrize("M,F,K", [(1024, 672, 1024), (4096, 2688, 1024), (300, 136, 128), (20000, 1408, 256),
                                   (2048, 5632, 2048)])  # Llama-1B gate|up
def test_gemm_pp_swiglu(M, F, K):
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(2 * F, K, device=DEV) * 0.05).bfloat16()
    gu, act = G.gemm_pp_swiglu(x, w)
    ref = x.float() @ w.float().t()
    assert rel(gu, ref) < 5e-3
    g, u = gu[:, :F].float(), gu[:, F:].float()  # act is computed from the rounded gate / up
    assert rel(act, torch.nn.functional.silu(g) * u) < 5e-3


@pytest.mark.parametrize("M,F,K", [(1024, 672, 1024), (4096, 2688, 1024), (300, 136, 128), (20000, 1408, 256),
                                   (2048, 5632, 2048)])  # Llama-1B down dgrad
def test_gemm_pp_dswiglu(M, F, K):
    gu = torch.randn(M, 2 * F, device=DEV).bfloat16()
    dy = torch.randn(M, K, device=DEV).bfloat16()
    wdt = (torch.randn(F, K, device=DEV) * 0.05).bfloat16()
    dgu = G.gemm_pp_dswiglu(dy, wdt, gu)
    dact = dy.float() @ wdt.float().t()
    g, u = gu[:, :F].float(), gu[:, F:].float()
    sg = torch.sigmoid(g)
    ref = torch.cat([dact * u * sg * (1 + g * (1 - sg)), dact * g * sg], 1)
    assert rel(dgu, ref) < 5e-3


def _fused_vs_chain(fused: bool, seed=0):
    """One Llama-150M-shaped MLP + q|k|v block through the model's op path with the fused epilogues
    on or off; returns outputs and gradients."""
    torch.manual_seed(seed)
    M, d, F, T, nh, hd = 2048, 256, 704, 512, 4, 64
    y = (torch.randn(M, d, device=DEV) * 0.5).bfloat16().requires_grad_(True)
    w_gu = (torch.randn(2 * F, d, device=DEV) * 0.05).bfloat16()
    w_dn = (torch.randn(d, F, device=DEV) * 0.05).bfloat16()
    w_qkv = (torch.randn(3 * nh * hd, d, device=DEV) * 0.05).bfloat16()
    g_gu, g_dn, g_qkv = (torch.zeros(w.shape, device=DEV) for w in (w_gu, w_dn, w_qkv))
    wt_gu, wt_dn, wt_qkv = w_gu.t().contiguous(), w_dn.t().contiguous(), w_qkv.t().contiguous()
    cos, sin = ops.rope_cache(T, hd, 10000.0, None, DEV)
    ops.set_fused_epilogues(rope=fused, mlp=fused)
    try:
        if fused:
            assert ops.mlp_fused_supported(y, w_gu, wt_gu, w_dn, wt_dn)
            m = ops.mlp_fused(y, w_gu, g_gu, wt_gu, w_dn, g_dn, wt_dn)
            assert ops.linear_rope_supported(y, w_qkv, wt_qkv, hd, 2 * nh * hd)
            qkv = ops.linear_rope(y, w_qkv, g_qkv, wt_qkv, cos, sin, T, hd, 2 * nh * hd)
            o = ops.attention(qkv, cos, sin, M // T, T, nh, nh, hd, inplace=True, rotated=True)
        else:
            act = ops.swiglu(ops.linear(y, w_gu, g_gu, wt_gu))
            m = ops.linear(act, w_dn, g_dn, wt_dn)
            qkv = ops.linear(y, w_qkv, g_qkv, wt_qkv)
            o = ops.attention(qkv, cos, sin, M // T, T, nh, nh, hd, inplace=True)
        loss = (m.float() * torch.linspace(-1, 1, d, device=DEV)).sum() + (o.float() ** 2).mean() * 100
        loss.backward()
    finally:
        ops.set_fused_epilogues(rope=True, mlp=True)
    return m.detach(), o.detach(), y.grad, g_gu, g_dn, g_qkv


def test_fused_mlp_and_rope_match_unfused_chain():
    f = _fused_vs_chain(True)
    u = _fused_vs_chain(False)
    for name, a, b in zip(["m", "o", "dy", "g_gu", "g_dn", "g_qkv"], f, u):
        assert rel(a, b) < 1e-2, name


def test_proj_gemm_switch_routes_to_own_kernel():
    """'pp' routes the plain projection products to gemm_pp (bitwise equal to a direct call); the
    default 'blas' uses torch.mm (hipBLASLt)."""
    x = torch.randn(1024, 512, device=DEV).bfloat16()
    w = (torch.randn(768, 512, device=DEV) * 0.05).bfloat16()
    assert ops.proj_gemm() == "blas"
    assert torch.equal(ops.mm_nt(x, w), torch.mm(x, w.t()))
    ops.set_proj_gemm("pp")
    try:
        assert torch.equal(ops.mm_nt(x, w), G.gemm_pp(x, w))
    finally:
        ops.set_proj_gemm("blas")


@pytest.mark.parametrize("proj", ["blas", "pp"])
def test_model_step_fused_vs_unfused(proj):
    """A 2-layer Llama forward+backward: the fused-epilogue path (default) and the unfused path give
    the same loss and gradients to bf16 tolerance, with either plain-GEMM backend."""
    from nanodiloco_amd.config import LlamaConfig
    from nanodiloco_amd.models import LlamaForCausalLM
    cfg = LlamaConfig(vocab_size=4096, hidden_size=256, intermediate_size=704, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=4, max_position_embeddings=512)
    ids = torch.randint(0, cfg.vocab_size, (4, 512), device=DEV)
    out = {}
    ops.set_proj_gemm(proj)
    try:
        for fused in (True, False):
            ops.set_fused_epilogues(rope=fused, mlp=fused)
            m = LlamaForCausalLM(cfg, DEV, torch.bfloat16).init_weights(3)
            loss = m(ids, labels=ids).loss
            loss.backward()
            out[fused] = (loss.detach().float(), m.store.grad.clone())
    finally:
        ops.set_fused_epilogues(rope=True, mlp=True)
        ops.set_proj_gemm("blas")
    assert abs(out[True][0].item() - out[False][0].item()) < 2e-3 * abs(out[False][0].item())
    assert rel(out[True][1], out[False][1]) < 2e-2
