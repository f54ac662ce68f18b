"""fp8 inner step (BASELINE config 5): quantiser numerics, fp8 linear vs fp32, fp8 training tracks bf16."""
import pytest
import torch

from nanodiloco_amd import ops
from nanodiloco_amd.config import LlamaConfig
from nanodiloco_amd.models import LlamaForCausalLM
from nanodiloco_amd.optim import FlatAdamW
from nanodiloco_amd.ops import fp8

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu(hip_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.set_backend("hip")
    torch.manual_seed(0)
    yield
    ops.set_backend("auto")


@pytest.mark.parametrize("fmt", [fp8.E4M3, fp8.E5M2])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n", [4096 * 8, 1000 * 7 + 3])
def test_cast_matches_torch(fmt, dt, n):
    x = (torch.randn(n, device="cuda") * 3).to(dt)
    x[5] = 1e6  # saturates
    scale = torch.tensor([37.5], device="cuda")
    amax = torch.zeros(fp8.AMAX_PARTS, device="cuda")
    q = fp8.cast(x, scale, fmt, amax)
    ref = (x.float() * 37.5).clamp(-fp8.FMAX[fmt], fp8.FMAX[fmt]).to(fp8.TORCH_DT[fmt])
    assert q.dtype == fp8.TORCH_DT[fmt]
    mism = (q.view(torch.uint8) != ref.view(torch.uint8)).sum().item()
    assert mism == 0, mism
    assert amax.max().item() == x.float().abs().max().item()


@pytest.mark.parametrize("fmt", [fp8.E4M3, fp8.E5M2])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_cast_t_matches_torch(fmt, dt):
    x = (torch.randn(192, 320, device="cuda") * 2).to(dt)
    scale = torch.tensor([11.0], device="cuda")
    amax = torch.zeros(fp8.AMAX_PARTS, device="cuda")
    q, qt = fp8.cast_t(x, scale, fmt, amax)
    ref = (x.float() * 11.0).clamp(-fp8.FMAX[fmt], fp8.FMAX[fmt]).to(fp8.TORCH_DT[fmt])
    assert torch.equal(q.view(torch.uint8), ref.view(torch.uint8))
    assert torch.equal(qt.view(torch.uint8), ref.t().contiguous().view(torch.uint8))
    assert amax.max().item() == x.float().abs().max().item()
    # strided rows (a column slice of a wider buffer)
    big = torch.randn(128, 256, device="cuda").to(dt)
    q2, qt2 = fp8.cast_t(big[:, 64:192], scale, fmt)
    ref2 = (big[:, 64:192].float() * 11.0).clamp(-fp8.FMAX[fmt], fp8.FMAX[fmt]).to(fp8.TORCH_DT[fmt])
    assert torch.equal(qt2.view(torch.uint8), ref2.t().contiguous().view(torch.uint8))


@pytest.mark.parametrize("wgrad_fp8", [True, False])
def test_fp8_linear_close_to_fp32(wgrad_fp8):
    M, N, K = 2048, 1536, 1024
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    gw = torch.zeros(N, K, device="cuda")
    lin = fp8.Fp8Linears("cuda", wgrad_fp8=wgrad_fp8)
    xr = x.clone().requires_grad_(True)
    y = lin("l", xr, w, gw, version=0)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    y.backward(dy)
    y_ref = x.float() @ w.float().t()
    dx_ref = dy.float() @ w.float()
    gw_ref = dy.float().t() @ x.float()
    rel = lambda a, b: ((a.float() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(y, y_ref) < 6e-2
    assert rel(xr.grad, dx_ref) < 1e-1
    assert rel(gw, gw_ref) < (8e-2 if wgrad_fp8 else 1e-2)
    # delayed scaling: the recipe saw both tensors and produces finite scales
    lin.recipe.update()
    assert torch.isfinite(lin.recipe.scale[:2]).all() and (lin.recipe.scale[:2] > 0).all()


def test_fp8_training_tracks_bf16():
    cfg = LlamaConfig.from_dict(dict(hidden_size=256, intermediate_size=768, num_attention_heads=4,
                                     num_key_value_heads=4, num_hidden_layers=2, vocab_size=512))
    ids = torch.randint(0, 512, (8, 256), device="cuda")
    losses = {}
    for use_fp8 in (False, True):
        m = LlamaForCausalLM(cfg, "cuda", torch.bfloat16, fp8=use_fp8).init_weights(5)
        opt = FlatAdamW(m.store, lr=3e-3)
        ls = []
        for _ in range(30):
            out = m(ids, labels=ids)
            out.loss.backward()
            opt.step()
            if m.fp8 is not None:
                m.fp8.recipe.update()
            m.store.zero_grad()
            ls.append(out.loss.item())
        losses[use_fp8] = ls
    b, f = losses[False], losses[True]
    assert f[-1] < 0.5 * f[0], f  # fp8 model memorises the batch
    assert abs(f[-1] - b[-1]) < 0.15 * b[0], (b[-1], f[-1])
