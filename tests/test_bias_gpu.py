"""Systematic-bias checks of the HIP kernels.

The per-kernel tests (test_kernels_gpu.py) bound the relative Frobenius error, which bf16 rounding
alone puts at 0.3-3 %: a kernel that scaled its output by 0.99 would still pass them.  Here each
output is projected onto its fp32 reference:

    beta = <out - ref, ref> / <ref, ref>

Unbiased rounding noise averages out in that projection (|beta| ~ 1e-5 at these sizes), while a
1 % scale error gives beta = -1e-2; the threshold is 1e-3.  The model-level test also requires the
HIP bf16 gradient to be no further from the fp32 reference than stock PyTorch ops in bf16 are
(same weights, same batch), so the hand-written kernels lose nothing against the library path.
"""
import pytest
import torch

from nanodiloco_amd import ops
from nanodiloco_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
BETA_MAX = 1e-3


@pytest.fixture(autouse=True)
def _hip(hip_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.set_backend("hip")
    torch.manual_seed(0)
    yield
    ops.set_backend("auto")


def beta(out, want):
    out, want = out.double().flatten(), want.double().flatten()
    return (torch.dot(out - want, want) / torch.dot(want, want)).item()


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("B,T,nh,nkv", [(8, 1024, 16, 16), (4, 1024, 32, 4)])
def test_attention_unbiased(B, T, nh, nkv):
    """Flash attention fwd / dQ / dK / dV at the Llama-150M and Llama-1B (GQA 32/4) shapes."""
    from nanodiloco_amd.ops.attention import rope_cache

    hd = 64
    qkv = torch.randn(B * T, (nh + 2 * nkv) * hd, device=DEV).bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, DEV)
    x = qkv.clone().requires_grad_(True)
    o = ops.attention(x, cos, sin, B, T, nh, nkv, hd)
    xr = qkv.float().requires_grad_(True)
    q, k, v = ref.split_qkv(xr, B, T, nh, nkv, hd)
    orf = ref.causal_attention(ref.apply_rope(q, cos, sin), ref.apply_rope(k, cos, sin), v)
    orf = orf.transpose(1, 2).reshape(B * T, nh * hd)
    do = torch.randn_like(orf).bfloat16()
    o.backward(do)
    orf.backward(do.float())
    nq, nk = nh * hd, nkv * hd
    g, gr = x.grad.float(), xr.grad
    parts = {"o": (o, orf.detach()), "dq": (g[:, :nq], gr[:, :nq]), "dk": (g[:, nq:nq + nk], gr[:, nq:nq + nk]),
             "dv": (g[:, nq + nk:], gr[:, nq + nk:])}
    for name, (a, b) in parts.items():
        assert abs(beta(a, b)) < BETA_MAX, (name, beta(a, b))


def test_rmsnorm_swiglu_unbiased():
    rows, cols, F, eps = 4096, 1024, 2688, 1e-5
    h = torch.randn(rows, cols, device=DEV)
    w = 1 + 0.1 * torch.randn(cols, device=DEV)
    gw = torch.zeros(cols, device=DEV)
    hx = h.clone().requires_grad_(True)
    hr = h.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y = ops.rmsnorm(hx, w, gw, eps, torch.bfloat16)
    yr = wr * (hr * torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + eps))
    dy = torch.randn(rows, cols, device=DEV).bfloat16()
    y.backward(dy)
    yr.backward(dy.float())
    for name, a, b in [("y", y, yr.detach()), ("dx", hx.grad, hr.grad), ("dw", gw, wr.grad)]:
        assert abs(beta(a, b)) < BETA_MAX, (name, beta(a, b))

    gu = torch.randn(rows, 2 * F, device=DEV).bfloat16().requires_grad_(True)
    gr = gu.detach().float().requires_grad_(True)
    s = ops.swiglu(gu)
    sr = ref.swiglu(gr)
    ds = torch.randn(rows, F, device=DEV).bfloat16()
    s.backward(ds)
    sr.backward(ds.float())
    for name, a, b in [("swiglu", s, sr.detach()), ("dswiglu", gu.grad, gr.grad)]:
        assert abs(beta(a, b)) < BETA_MAX, (name, beta(a, b))


def test_lm_head_ce_unbiased():
    n, d, V = 2048, 1024, 32000
    y = (0.5 * torch.randn(n, d, device=DEV)).bfloat16().requires_grad_(True)
    W = (0.05 * torch.randn(V, d, device=DEV)).bfloat16()
    gW = torch.zeros(V, d, device=DEV)
    tgt = torch.randint(0, V, (n,), device=DEV)
    loss = ops.lm_head_ce(y, W, gW, tgt, loss_scale=1.0)
    loss.backward()
    yr = y.detach().float().requires_grad_(True)
    Wr = W.float().requires_grad_(True)
    lr_ = torch.nn.functional.cross_entropy(yr @ Wr.t(), tgt)
    lr_.backward()
    assert abs(loss.item() - lr_.item()) < 1e-3 * abs(lr_.item())
    for name, a, b in [("dy", y.grad, yr.grad), ("dW", gW, Wr.grad)]:
        assert abs(beta(a, b)) < BETA_MAX, (name, beta(a, b))


def _model_grad(cfg, backend, ids, dtype):
    from nanodiloco_amd.models import LlamaForCausalLM

    ops.set_backend(backend)
    m = LlamaForCausalLM(cfg, DEV, dtype).init_weights(3)
    out = m(ids, labels=ids)
    out.loss.backward()
    torch.cuda.synchronize()
    return out.loss.item(), m.store.grad.clone()


def test_model_gradient_unbiased_and_no_worse_than_torch_bf16():
    """Whole 150M-width model (2 layers, d = 1024, 16 heads, V = 32000): the HIP bf16 gradient is
    unbiased against the fp32 PyTorch path and at most 1.25x as far from it as PyTorch's own bf16
    ops are (HIP fp32 residual stream + fp32 accumulation everywhere should make it closer)."""
    from nanodiloco_amd.config import LlamaConfig

    cfg = LlamaConfig.from_dict(dict(hidden_size=1024, intermediate_size=2688, num_attention_heads=16,
                                     num_key_value_heads=16, num_hidden_layers=2, vocab_size=32000,
                                     rms_norm_eps=1e-5))
    ids = torch.randint(0, 32000, (4, 1024), device=DEV)
    l32, g32 = _model_grad(cfg, "torch", ids, torch.float32)
    lt16, gt16 = _model_grad(cfg, "torch", ids, torch.bfloat16)
    lh, gh = _model_grad(cfg, "hip", ids, torch.bfloat16)
    assert abs(lh - l32) <= max(1.25 * abs(lt16 - l32), 2e-3 * abs(l32)), (lh, lt16, l32)
    assert abs(beta(gh, g32)) < 5 * BETA_MAX, beta(gh, g32)
    assert rel(gh, g32) <= 1.25 * rel(gt16, g32) + 1e-3, (rel(gh, g32), rel(gt16, g32))
