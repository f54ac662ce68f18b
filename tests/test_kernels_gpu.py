"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op (T3)."""
import math

import pytest
import torch

from nanodiloco_amd import ops
from nanodiloco_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True)
def _hip(hip_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.set_backend("hip")
    torch.manual_seed(0)
    yield
    ops.set_backend("auto")


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


# ----------------------------------------------------------------------------------- rmsnorm
@pytest.mark.parametrize("cols", [128, 1024, 2048])
@pytest.mark.parametrize("residual", [False, True])
def test_rmsnorm_fwd_bwd(cols, residual):
    rows, eps = 1000, 1e-5
    h = torch.randn(rows, cols, device=DEV)
    a = torch.randn(rows, cols, device=DEV).bfloat16()
    w = (1 + 0.1 * torch.randn(cols, device=DEV))
    gw = torch.zeros(cols, device=DEV)
    hr = h.clone().requires_grad_(True)
    ar = a.clone().float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    hh = hr + ar if residual else hr
    yr = wr * (hh * torch.rsqrt(hh.pow(2).mean(-1, keepdim=True) + eps))
    hx = h.clone().requires_grad_(True)
    ax = a.clone().requires_grad_(True)
    if residual:
        y, hn = ops.add_rmsnorm(hx, ax, w, gw, eps, torch.bfloat16)
        assert rel(hn, (h + a.float())) < 1e-6
    else:
        y = ops.rmsnorm(hx, w, gw, eps, torch.bfloat16)
    assert y.dtype == torch.bfloat16
    assert rel(y, yr) < 5e-3
    dy = torch.randn(rows, cols, device=DEV)
    (yr * dy).sum().backward()
    (y.float() * dy.bfloat16().float()).sum().backward()
    assert rel(hx.grad, hr.grad) < 1e-2
    assert rel(gw, wr.grad) < 1e-2
    if residual:
        assert rel(ax.grad, ar.grad) < 1e-2


def test_rmsnorm_res_fused_residual_grad():
    """rmsnorm_res: the residual gradient enters the HIP backward kernel as ``dres``; compare with the
    plain fp32 PyTorch reference where autograd sums the two uses of x."""
    rows, cols, eps = 1000, 1024, 1e-5
    x = torch.randn(rows, cols, device=DEV)
    w = 1 + 0.1 * torch.randn(cols, device=DEV)
    up = torch.randn(rows, cols, device=DEV).bfloat16()
    ur = torch.randn(rows, cols, device=DEV)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = wr * (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + eps))
    ((yr * up.float()).sum() + (xr * ur).sum()).backward()
    xx = x.clone().requires_grad_(True)
    gw = torch.zeros(cols, device=DEV)
    y, h = ops.rmsnorm_res(xx, w, gw, eps, torch.bfloat16)
    assert y.dtype == torch.bfloat16 and h.data_ptr() == xx.data_ptr()
    ((y.float() * up.float()).sum() + (h * ur).sum()).backward()
    assert rel(y, yr) < 5e-3
    assert rel(xx.grad, xr.grad) < 1e-2
    assert rel(gw, wr.grad) < 1e-2


@pytest.mark.parametrize("cols", [1024, 2048])
def test_add_rmsnorm_bf16_residual(cols):
    """bf16 residual stream (--residual-dtype bf16): h_new is the RNE-rounded h + a (bitwise), y / dh / da /
    dw match an fp32 reference computed from that rounded h_new, and the residual gradient IS the branch
    gradient (one bf16 tensor)."""
    rows, eps = 1000, 1e-5
    h = torch.randn(rows, cols, device=DEV).bfloat16()
    a = torch.randn(rows, cols, device=DEV).bfloat16()
    w = 1 + 0.1 * torch.randn(cols, device=DEV)
    dres = torch.randn(rows, cols, device=DEV).bfloat16()
    dy = torch.randn(rows, cols, device=DEV).bfloat16()
    hn_ref = (h.float() + a.float()).bfloat16()
    xr = hn_ref.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = wr * (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + eps))
    ((yr * dy.float()).sum() + (xr * dres.float()).sum()).backward()
    hx, ax = h.clone().requires_grad_(True), a.clone().requires_grad_(True)
    gw = torch.zeros(cols, device=DEV)
    y, hn = ops.add_rmsnorm(hx, ax, w, gw, eps, torch.bfloat16)
    assert hn.dtype == torch.bfloat16 and torch.equal(hn, hn_ref)
    assert rel(y, yr) < 5e-3
    dh, da = torch.autograd.grad((y, hn), (hx, ax), (dy, dres))
    assert dh.dtype == torch.bfloat16 and da.dtype == torch.bfloat16
    assert dh.data_ptr() == da.data_ptr()  # one store serves both
    assert rel(dh, xr.grad) < 1e-2
    gw2 = torch.zeros(cols, device=DEV)
    hx2, ax2 = h.clone().requires_grad_(True), a.clone().requires_grad_(True)
    y2, _ = ops.add_rmsnorm(hx2, ax2, w, gw2, eps, torch.bfloat16)
    (y2.float() * dy.float()).sum().backward()
    wr2 = w.clone().requires_grad_(True)
    x2 = hn_ref.float()
    (wr2 * (x2 * torch.rsqrt(x2.pow(2).mean(-1, keepdim=True) + eps)) * dy.float()).sum().backward()
    assert rel(gw2, wr2.grad) < 1e-2


def test_rmsnorm_res_bf16_residual():
    """First norm on a bf16 residual stream: bf16 dres in, bf16 dx out, fp32 reference."""
    rows, cols, eps = 1000, 1024, 1e-5
    x = torch.randn(rows, cols, device=DEV).bfloat16()
    w = 1 + 0.1 * torch.randn(cols, device=DEV)
    up = torch.randn(rows, cols, device=DEV).bfloat16()
    ur = torch.randn(rows, cols, device=DEV).bfloat16()
    xr = x.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = wr * (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + eps))
    ((yr * up.float()).sum() + (xr * ur.float()).sum()).backward()
    xx = x.clone().requires_grad_(True)
    gw = torch.zeros(cols, device=DEV)
    y, h = ops.rmsnorm_res(xx, w, gw, eps, torch.bfloat16)
    torch.autograd.backward((y, h), (up, ur))
    assert xx.grad.dtype == torch.bfloat16
    assert rel(y, yr) < 5e-3
    assert rel(xx.grad, xr.grad) < 1e-2
    assert rel(gw, wr.grad) < 1e-2


# ----------------------------------------------------------------------------------- rope
@pytest.mark.parametrize("hd,nh,nkv", [(64, 4, 4), (128, 4, 2), (32, 4, 1)])
def test_rope_inplace_matches_reference(hd, nh, nkv, hip_lib):
    from nanodiloco_amd.ops import _ext
    from nanodiloco_amd.ops.attention import _rope, rope_cache

    B, T = 2, 96
    ld = (nh + 2 * nkv) * hd
    qkv = torch.randn(B * T, ld, device=DEV).bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, DEV)
    out = qkv.clone()
    _rope(out, cos, sin, B, T, nh, nkv, hd, inverse=False)
    q, k, v = ref.split_qkv(qkv.float(), B, T, nh, nkv, hd)
    qr = ref.apply_rope(q, cos, sin)
    kr = ref.apply_rope(k, cos, sin)
    q2, k2, v2 = ref.split_qkv(out.float(), B, T, nh, nkv, hd)
    assert rel(q2, qr) < 5e-3 and rel(k2, kr) < 5e-3
    assert torch.equal(v2, v)
    back = out.clone()
    _rope(back, cos, sin, B, T, nh, nkv, hd, inverse=True)
    assert rel(back, qkv) < 1e-2


# ----------------------------------------------------------------------------------- swiglu
@pytest.mark.parametrize("F", [512, 2688])
def test_swiglu(F):
    n = 777
    gu = torch.randn(n, 2 * F, device=DEV).bfloat16().requires_grad_(True)
    gr = gu.detach().float().requires_grad_(True)
    y = ops.swiglu(gu)
    yr = ref.swiglu(gr)
    assert rel(y, yr) < 5e-3
    dy = torch.randn(n, F, device=DEV).bfloat16()
    y.backward(dy)
    yr.backward(dy.float())
    assert rel(gu.grad, gr.grad) < 1e-2


# ----------------------------------------------------------------------------------- embedding
@pytest.mark.parametrize("odt", [torch.float32, torch.bfloat16])
def test_embedding(odt):
    """fp32 rows, or bf16 rows (RNE in the gather) for the bf16 residual stream with a bf16 dy backward."""
    V, d, n = 1000, 256, 4096
    W = torch.randn(V, d, device=DEV)
    gW = torch.zeros(V, d, device=DEV)
    ids = torch.randint(0, V, (4, n // 4), device=DEV)
    out = ops.embedding(ids, W, gW, out_dtype=odt)
    assert out.dtype == odt and torch.equal(out, W[ids.reshape(-1)].to(odt))
    dy = torch.randn(n, d, device=DEV).to(odt)
    out.backward(dy)
    ref_g = torch.zeros(V, d, device=DEV).index_add_(0, ids.reshape(-1), dy.float())
    assert rel(gW, ref_g) < 1e-6


# ----------------------------------------------------------------------------------- fused lm_head + CE
@pytest.mark.parametrize("V", [32000, 1000, 50257])
def test_lm_head_ce(V):
    n, d = 640, 256
    y = (0.5 * torch.randn(n, d, device=DEV)).bfloat16().requires_grad_(True)
    W = (0.05 * torch.randn(V, d, device=DEV)).bfloat16()
    gW = torch.zeros(V, d, device=DEV)
    tgt = torch.randint(0, V, (n,), device=DEV)
    tgt[::7] = -100
    scale = 0.25
    loss = ops.lm_head_ce(y, W, gW, tgt, loss_scale=scale, chunk_rows=256)
    loss.backward()
    yr = y.detach().float().requires_grad_(True)
    Wr = W.float().requires_grad_(True)
    lr_ = torch.nn.functional.cross_entropy(yr @ Wr.t(), tgt, ignore_index=-100)
    (lr_ * scale).backward()
    assert abs(loss.item() - lr_.item()) < 2e-3 * max(1.0, abs(lr_.item()))
    assert rel(y.grad, yr.grad) < 2e-2
    assert rel(gW, Wr.grad) < 2e-2


# ----------------------------------------------------------------------------------- attention
def _attn_ref(qkv, cos, sin, B, T, nh, nkv, hd):
    q, k, v = ref.split_qkv(qkv.float(), B, T, nh, nkv, hd)
    q = ref.apply_rope(q, cos, sin)
    k = ref.apply_rope(k, cos, sin)
    o = ref.causal_attention(q, k, v)
    return o.transpose(1, 2).reshape(B * T, nh * hd)


@pytest.mark.parametrize("B,T,nh,nkv,hd", [
    (2, 64, 2, 2, 64), (2, 200, 4, 4, 64), (1, 1024, 2, 2, 64), (2, 256, 4, 1, 64),
    (2, 130, 4, 4, 32), (1, 300, 2, 1, 128), (1, 2048, 1, 1, 64),
    (8, 1024, 16, 16, 64),  # Llama-150M bench shape (batch 64 -> 8: same per-head work, smaller grid)
    (4, 1024, 32, 4, 64),   # Llama-1B GQA 32/4
    (1, 8192, 2, 1, 64),    # long context: 8k tokens, GQA
    (1, 4096, 2, 2, 128),
])
def test_flash_attention_fwd_bwd(B, T, nh, nkv, hd):
    from nanodiloco_amd.ops.attention import rope_cache

    ld = (nh + 2 * nkv) * hd
    qkv = torch.randn(B * T, ld, device=DEV).bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, DEV)
    x = qkv.clone().requires_grad_(True)
    o = ops.attention(x, cos, sin, B, T, nh, nkv, hd)
    xr = qkv.float().requires_grad_(True)
    orf = _attn_ref(xr, cos, sin, B, T, nh, nkv, hd)
    assert o.shape == (B * T, nh * hd)
    assert rel(o, orf) < 1e-2, rel(o, orf)
    do = torch.randn_like(orf)
    o.backward(do.bfloat16())
    orf.backward(do.bfloat16().float())
    g, gr = x.grad.float(), xr.grad
    nq, nk = nh * hd, nkv * hd
    assert rel(g[:, :nq], gr[:, :nq]) < 3e-2, ("dq", rel(g[:, :nq], gr[:, :nq]))
    assert rel(g[:, nq:nq + nk], gr[:, nq:nq + nk]) < 3e-2, ("dk", rel(g[:, nq:nq + nk], gr[:, nq:nq + nk]))
    assert rel(g[:, nq + nk:], gr[:, nq + nk:]) < 3e-2, ("dv", rel(g[:, nq + nk:], gr[:, nq + nk:]))


def test_flash_attention_softmax_spike():
    """Force a large max jump mid-sequence (online-softmax rescale path, rule 26)."""
    from nanodiloco_amd.ops.attention import rope_cache

    B, T, nh, nkv, hd = 1, 512, 1, 1, 64
    ld = (nh + 2 * nkv) * hd
    qkv = torch.randn(B * T, ld, device=DEV)
    qkv[300, nh * hd:(nh + nkv) * hd] *= 30.0  # one key row with a huge score for many queries
    qkv = qkv.bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, DEV)
    o = ops.attention(qkv, cos, sin, B, T, nh, nkv, hd)
    orf = _attn_ref(qkv, cos, sin, B, T, nh, nkv, hd)
    assert rel(o, orf) < 1e-2


# ----------------------------------------------------------------------------------- optimizers
def test_adamw_matches_torch():
    n = 100_003 + 64 - (100_003 % 64)
    p0 = torch.randn(n, device=DEV)
    grads = [torch.randn(n, device=DEV) * 3 for _ in range(3)]
    # torch reference
    p = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([p], lr=1e-3, weight_decay=0.01)
    for g in grads:
        p.grad = g.clone()
        torch.nn.utils.clip_grad_norm_([p], 1.0)
        opt.step()
    # ours
    master = p0.clone()
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    sh = torch.zeros(n, device=DEV, dtype=torch.bfloat16)
    norm = torch.zeros(1, device=DEV)
    for i, g in enumerate(grads):
        ops.adamw_step(master, g.clone(), m, v, sh, i + 1, 1e-3, (0.9, 0.999), 1e-8, 0.01, 1.0, norm_out=norm)
    assert (master - p.detach()).abs().max().item() < 1e-5
    assert abs(norm.item() - grads[-1].norm().item()) / grads[-1].norm().item() < 1e-4
    assert torch.equal(sh, master.bfloat16())


@pytest.mark.parametrize("comm", [torch.float32, torch.bfloat16])
def test_outer_nesterov_matches_torch_sgd(comm):
    n = 4096
    sync = torch.randn(n, device=DEV)
    local = sync - 0.01 * torch.randn(n, device=DEV)
    # torch reference: param = sync, grad = avg delta, SGD nesterov
    p = torch.nn.Parameter(sync.clone())
    opt = torch.optim.SGD([p], lr=0.7, momentum=0.9, nesterov=True)
    delta = torch.empty(n, device=DEV, dtype=comm)
    ops.pseudograd(sync, local, delta)
    p.grad = delta.float().clone()
    opt.step()
    master = local.clone()
    s2 = sync.clone()
    mom = torch.zeros(n, device=DEV)
    ops.outer_nesterov(master, s2, delta, mom, None, 1.0, 0.7, 0.9, True)
    assert (master - p.detach()).abs().max().item() < 1e-6
    assert torch.equal(master, s2)


# ----------------------------------------------------------------------------------- wgrad GEMM
@pytest.mark.parametrize("M,N,K", [(3072, 1024, 4096), (1024, 1024, 32768), (1000, 264, 777), (32000, 1024, 2048),
                                   (128, 512, 64), (5376, 1024, 65536), (1024, 2688, 16640),
                                   # Llama-1B: q|k|v, gate|up, down, lm head
                                   (2560, 2048, 8192), (11264, 2048, 4096), (2048, 5632, 4096), (32000, 2048, 2048)])
@pytest.mark.parametrize("variant", ["", "dma0", "dmas", "b"])
def test_wgrad_gemm(M, N, K, variant, monkeypatch):
    monkeypatch.setenv("ND_WGRAD_VARIANT", variant)
    from nanodiloco_amd.ops.gemm import wgrad
    dy = torch.randn(K, M, device=DEV).bfloat16()
    x = torch.randn(K, N, device=DEV).bfloat16()
    gw0 = torch.randn(M, N, device=DEV)
    gw = gw0.clone()
    wgrad(gw, dy, x)
    ref_ = gw0 + dy.float().t() @ x.float()
    assert rel(gw, ref_) < 1e-5, rel(gw, ref_)
    gw2 = gw0.clone()
    wgrad(gw2, dy, x)
    assert torch.equal(gw, gw2)  # deterministic (no atomics)


@pytest.mark.parametrize("variant", ["", "dma0", "dmas", "b"])
def test_wgrad_no_empty_split_with_poisoned_slabs(variant, monkeypatch):
    """K = 41 * 64 over 16 output tiles: rounding the per-split K chunk up to whole tiles would leave the
    last split empty; its slab plane must not be summed stale (the workspace is NaN-poisoned first)."""
    monkeypatch.setenv("ND_WGRAD_VARIANT", variant)
    from nanodiloco_amd.ops import gemm as G
    M = N = 1024
    K = 41 * 64
    G._workspace(torch.device(DEV), 16 * M * N).fill_(float("nan"))
    dy = torch.randn(K, M, device=DEV).bfloat16()
    x = torch.randn(K, N, device=DEV).bfloat16()
    gw = torch.zeros(M, N, device=DEV)
    G.wgrad(gw, dy, x)
    assert torch.isfinite(gw).all()
    assert rel(gw, dy.float().t() @ x.float()) < 1e-5


@pytest.mark.parametrize("shapes,K", [(((1024, 2688), (5376, 1024)), 16384),   # Llama-150M down + gate|up
                                      (((3072, 1024), (1024, 1024)), 8192),    # q|k|v + o
                                      (((2048, 5632), (11264, 2048)), 4096),   # Llama-1B down + gate|up (not grouped)
                                      (((1000, 1032), (520, 2048)), 41 * 64)])  # partial tiles, K tail
def test_wgrad_grouped(shapes, K):
    """Two weight gradients in one grouped launch (nd_wgrad2) against fp32 references; run twice with
    NaN-poisoned slabs in between (deterministic, no stale slab plane summed)."""
    from nanodiloco_amd.ops import gemm as G
    (M0, N0), (M1, N1) = shapes
    dy0, x0 = torch.randn(K, M0, device=DEV).bfloat16(), torch.randn(K, N0, device=DEV).bfloat16()
    dy1, x1 = torch.randn(K, M1, device=DEV).bfloat16(), torch.randn(K, N1, device=DEV).bfloat16()
    g0, g1 = torch.randn(M0, N0, device=DEV), torch.randn(M1, N1, device=DEV)
    r0, r1 = g0 + dy0.float().t() @ x0.float(), g1 + dy1.float().t() @ x1.float()
    S = ext_lib().nd_wgrad2_splits(M0, N0, M1, N1, K)
    if S == 0:  # the makespan model prefers two launches (Llama-1B MLP): nothing issued
        a0 = g0.clone()
        assert not G.wgrad2(a0, dy0, x0, g1.clone(), dy1, x1)
        assert torch.equal(a0, g0)
        return
    outs = []
    for _ in range(2):
        G._workspace(torch.device(DEV), 16 * (M0 * N0 + M1 * N1)).fill_(float("nan"))
        a0, a1 = g0.clone(), g1.clone()
        assert G.wgrad2(a0, dy0, x0, a1, dy1, x1)
        assert rel(a0, r0) < 1e-5 and rel(a1, r1) < 1e-5, (rel(a0, r0), rel(a1, r1))
        outs.append((a0, a1))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    if shapes[0] == (1024, 2688) and K == 16384:
        assert S == 2, S  # 44 + 84 tiles: 256 workgroups


def test_wgrad_grouped_refuses_mismatch():
    from nanodiloco_amd.ops import gemm as G
    dy0, x0 = torch.randn(512, 1024, device=DEV).bfloat16(), torch.randn(512, 1024, device=DEV).bfloat16()
    dy1, x1 = torch.randn(256, 1024, device=DEV).bfloat16(), torch.randn(256, 1024, device=DEV).bfloat16()
    g = torch.zeros(1024, 1024, device=DEV)
    assert not G.wgrad2(g, dy0, x0, g.clone(), dy1, x1)  # different K: not grouped, nothing issued
    assert g.abs().max().item() == 0


def ext_lib():
    from nanodiloco_amd.ops import _ext
    return _ext.lib()


def test_wgrad_strided_views():
    """Operands that are column slices of a wider buffer (fused q|k|v grads)."""
    from nanodiloco_amd.ops.gemm import wgrad
    K = 512
    big = torch.randn(K, 384, device=DEV).bfloat16()
    dy = big[:, 128:256]
    x = torch.randn(K, 256, device=DEV).bfloat16()
    gw = torch.zeros(128, 256, device=DEV)
    wgrad(gw, dy, x)
    assert rel(gw, dy.float().t() @ x.float()) < 1e-5


# ----------------------------------------------------------------------------------- attention rope modes
@pytest.mark.parametrize("hd,T", [(64, 200), (32, 130), (128, 96)])
def test_attention_raw_qkv_rope_mode1(hd, T):
    """Kernels applying RoPE on load (rope_mode 1 / fwd tables) on the raw projection output."""
    from nanodiloco_amd.ops import _ext
    from nanodiloco_amd.ops.attention import rope_cache
    B, nh, nkv = 2, 4, 2
    ld = (nh + 2 * nkv) * hd
    qkv = torch.randn(B * T, ld, device=DEV).bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, DEV)
    L = _ext.lib()
    s = _ext.stream_ptr(qkv.device)
    k, v = qkv[:, nh * hd:], qkv[:, (nh + nkv) * hd:]
    o = torch.empty(B * T, nh * hd, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, nh, T, device=DEV)
    _ext.check(L.nd_attn_fwd(qkv.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, nh, nkv, T,
                             hd, ld, nh * hd, cos.data_ptr(), sin.data_ptr(), hd ** -0.5, s), "fwd")
    xr = qkv.float().requires_grad_(True)
    orf = _attn_ref(xr, cos, sin, B, T, nh, nkv, hd)
    assert rel(o, orf) < 1e-2
    do = torch.randn_like(orf).bfloat16()
    orf.backward(do.float())
    delta = torch.empty(B, nh, T, device=DEV)
    _ext.check(L.nd_attn_bwd_pre(o.data_ptr(), do.data_ptr(), delta.data_ptr(), B, nh, T, hd, nh * hd, s), "pre")
    dqkv = torch.empty_like(qkv)
    dk, dv = dqkv[:, nh * hd:], dqkv[:, (nh + nkv) * hd:]
    _ext.check(L.nd_attn_bwd(qkv.data_ptr(), k.data_ptr(), v.data_ptr(), do.data_ptr(), lse.data_ptr(),
                             delta.data_ptr(), dqkv.data_ptr(), dk.data_ptr(), dv.data_ptr(), 0, B, nh, nkv, T, hd, ld,
                             nh * hd, cos.data_ptr(), sin.data_ptr(), hd ** -0.5, 1, s), "bwd")
    assert rel(dqkv, xr.grad) < 3e-2


def test_adamw_skip_nonfinite_on_device():
    n = 4096
    master = torch.randn(n, device=DEV)
    before = master.clone()
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    g = torch.randn(n, device=DEV)
    g[100] = float("inf")
    skipped = torch.zeros(1, dtype=torch.int32, device=DEV)
    ops.adamw_step(master, g, m, v, None, 1, 1e-3, skip_nonfinite=True, skipped=skipped)
    assert torch.equal(master, before) and int(skipped.item()) == 1


# ----------------------------------------------------------------------------------- transpose
@pytest.mark.parametrize("rows,cols", [(3072, 1024), (1024, 2688), (100, 72), (32000, 1024)])
def test_transpose_bf16(rows, cols):
    """W^T copies for the input-gradient GEMMs: exact (a permutation), edge tiles included."""
    w = torch.randn(rows, cols, device=DEV).bfloat16()
    out = torch.empty(cols, rows, device=DEV, dtype=torch.bfloat16)
    ops.transpose_into(out, w)
    assert torch.equal(out, w.t())


@pytest.mark.parametrize("rows", [1024, 700])
def test_colsum_add(rows):
    """RMSNorm dW partial-row reduction into the flat grad (fixed order, += into existing)."""
    from nanodiloco_amd.ops import _ext
    cols = 1024
    part = torch.randn(rows, cols, device=DEV)
    out = torch.randn(cols, device=DEV)
    ref_ = out.double() + part.double().sum(0)
    _ext.check(_ext.lib().nd_colsum_add(part.data_ptr(), out.data_ptr(), rows, cols, _ext.stream_ptr()), "colsum")
    assert rel(out, ref_) < 1e-6



@pytest.mark.parametrize("kv", [16, 4])
def test_attention_bwd_fused_stats_matches_separate(kv):
    """Row statistics computed inside the dQ kernel == the separate delta/statistics passes (up to
    the order of the delta summation), with GQA too."""
    from nanodiloco_amd.ops.attention import rope_cache, set_attn_fused_stats
    B, T, nh, hd = 2, 512, 16, 64
    qkv = (torch.randn(B * T, (nh + 2 * kv) * hd, device=DEV) * 0.5).bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, DEV)
    do = torch.randn(B * T, nh * hd, device=DEV).bfloat16()
    grads = []
    for fused in (False, True):
        set_attn_fused_stats(fused)
        try:
            x = qkv.clone().requires_grad_(True)
            o = ops.attention(x, cos, sin, B, T, nh, kv, hd)
            (g,) = torch.autograd.grad(o, x, do)
            grads.append(g.float())
        finally:
            set_attn_fused_stats(True)
    assert rel(grads[1], grads[0]) < 2e-3


@pytest.mark.parametrize("B,T,nh,nkv,hd,pads", [
    (3, 256, 4, 4, 64, (0, 37, 200)),        # fused backward (T % 64 == 0): dQ+stats, LDS-DMA dK/dV
    (2, 200, 4, 2, 64, (130, 5)),            # T % 64 != 0: register-staged kernels
    (4, 1024, 16, 16, 64, (0, 1, 511, 1000)),  # Llama-150M attention shape (batch reduced)
    (2, 1024, 32, 4, 64, (64, 700)),         # Llama-1B GQA 32/4
    (2, 130, 2, 1, 32, (17, 129)),
])
def test_flash_attention_left_padding_matches_sdpa_mask(B, T, nh, nkv, hd, pads):
    """Left-padded batches: the kernels' per-sequence key start against torch SDPA (fp32) with the
    boolean causal & padding mask HF builds from attention_mask (REF/nanodiloco/main.py:79-88,109);
    pad query rows are fully masked and output 0 on both sides.  Forward and all three gradients."""
    from nanodiloco_amd.ops.attention import key_start, rope_cache

    ld = (nh + 2 * nkv) * hd
    mask = torch.ones(B, T, dtype=torch.long, device=DEV)
    for b, p in enumerate(pads):
        mask[b, :p] = 0
    ks = key_start(mask)
    assert ks.tolist() == list(pads)
    qkv = torch.randn(B * T, ld, device=DEV).bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, DEV)
    x = qkv.clone().requires_grad_(True)
    o = ops.attention(x, cos, sin, B, T, nh, nkv, hd, kstart=ks)
    xr = qkv.float().requires_grad_(True)
    orf = ref.attention_block(xr, cos, sin, B, T, nh, nkv, hd, kstart=ks)
    assert torch.isfinite(o.float()).all()
    assert rel(o, orf) < 1e-2, rel(o, orf)
    pad_rows = (mask == 0).reshape(-1)
    assert (o[pad_rows] == 0).all()  # fully masked query rows
    do = torch.randn_like(orf)
    o.backward(do.bfloat16())
    orf.backward(do.bfloat16().float())
    g, gr = x.grad.float(), xr.grad
    assert torch.isfinite(g).all()
    nq, nk = nh * hd, nkv * hd
    assert rel(g[:, :nq], gr[:, :nq]) < 3e-2, ("dq", rel(g[:, :nq], gr[:, :nq]))
    assert rel(g[:, nq:nq + nk], gr[:, nq:nq + nk]) < 3e-2, ("dk", rel(g[:, nq:nq + nk], gr[:, nq:nq + nk]))
    assert rel(g[:, nq + nk:], gr[:, nq + nk:]) < 3e-2, ("dv", rel(g[:, nq + nk:], gr[:, nq + nk:]))
    # pad keys get no gradient from real queries, pad queries none at all
    assert (g[pad_rows] == 0).all()


def test_model_left_padded_hip_vs_torch():
    """The full model on the HIP path with a left-padded batch tracks the fp32 torch path."""
    from nanodiloco_amd.config import LlamaConfig
    from nanodiloco_amd.models import LlamaForCausalLM

    cfg = LlamaConfig.from_dict(dict(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                                     num_hidden_layers=2, vocab_size=1000))
    ids = torch.randint(0, 1000, (3, 128), device=DEV)
    mask = torch.ones_like(ids)
    mask[1, :40] = 0
    mask[2, :100] = 0
    labels = ids.clone()
    labels[mask == 0] = -100
    losses = []
    for backend, dt in (("hip", torch.bfloat16), ("torch", torch.float32)):
        ops.set_backend(backend)
        m = LlamaForCausalLM(cfg, DEV, dt).init_weights(0)
        losses.append(float(m(ids, labels=labels, attention_mask=mask).loss))
    ops.set_backend("hip")
    assert abs(losses[0] - losses[1]) < 2e-2 * abs(losses[1]), losses


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", ["repeated", "left_pad", "chunk_edges"])
def test_embedding_sorted_backward_deterministic(case, dt):
    """nd_embedding_bwd_sorted (stable argsort, 64-row chunks + ordered join of the runs that cross
    chunks) equals the index_add reference and is bitwise repeatable: heavily repeated ids (one id
    takes 25 % of the rows), a left-padded batch (6000 pad rows of one id, out-of-range ids skipped),
    and runs that end exactly on / one past chunk boundaries."""
    from nanodiloco_amd.ops import _ext
    from nanodiloco_amd.ops.embedding import sorted_bwd_workspace

    n, d, V = 8192, 1024, 5000
    ids = torch.randint(0, V, (n,), device=DEV)
    if case == "repeated":
        ids[::4] = 7
    elif case == "left_pad":
        ids[:6000] = 0
        ids[6000:6010] = V + 3  # out of range: skipped
    else:
        n = 64 * 37 + 5
        ids = torch.repeat_interleave(torch.arange(0, 200, device=DEV),
                                      torch.tensor([64, 1, 63, 128, 65, 127] * 33 + [5, 9], device=DEV))[:n]
        n = ids.numel()
    dy = torch.randn(n, d, device=DEV).to(dt)
    base = torch.randn(V, d, device=DEV)
    outs = []
    for _ in range(2):
        gW = base.clone()
        perm = torch.argsort(ids, stable=True)
        sid = ids.index_select(0, perm).contiguous()
        ws = sorted_bwd_workspace(n, d, DEV).fill_(float("nan"))  # partials must be fully written
        _ext.check(_ext.lib().nd_embedding_bwd_sorted(sid.data_ptr(), perm.data_ptr(), dy.data_ptr(), _ext.dtcode(dy),
                                                      gW.data_ptr(), ws.data_ptr(), n, d, V, _ext.stream_ptr()), "sorted")
        outs.append(gW)
    assert torch.equal(outs[0], outs[1])
    ok = (ids >= 0) & (ids < V)
    ref_gw = base.double().index_add_(0, ids[ok], dy[ok].double())  # bf16 dy: exact in double
    assert torch.allclose(outs[0].double(), ref_gw, atol=1e-3, rtol=1e-5)


def test_deterministic_mode_bitwise_repeatable_step():
    """--deterministic: two fwd+bwd passes of the model on the same batch give bitwise-identical
    loss and gradient buffers (no float atomics anywhere on the step)."""
    from nanodiloco_amd.config import LlamaConfig
    from nanodiloco_amd.models import LlamaForCausalLM

    ops.set_deterministic(True)
    try:
        cfg = LlamaConfig.from_dict(dict(hidden_size=512, intermediate_size=1024, num_attention_heads=8,
                                         num_hidden_layers=2, vocab_size=4096))
        m = LlamaForCausalLM(cfg, DEV, torch.bfloat16).init_weights(0)
        ids = torch.randint(0, 4096, (4, 512), device=DEV)
        ids[:, ::3] = 11  # repeated ids: many colliding embedding-gradient rows
        res = []
        for _ in range(2):
            m.store.zero_grad()
            out = m(ids, labels=ids)
            out.loss.backward()
            torch.cuda.synchronize()
            res.append((out.loss.detach().clone(), m.store.grad.clone()))
        assert torch.equal(res[0][0], res[1][0])
        bad = []
        for name in m.store.names:
            a, b = m.store.grad_view(name), None
            off = m.store.offsets[name] if hasattr(m.store, "offsets") else None
            ga = res[0][1]
            gb = res[1][1]
            va, vb = _store_view(m.store, ga, name), _store_view(m.store, gb, name)
            if not torch.equal(va, vb):
                bad.append((name, float((va - vb).abs().max())))
        assert not bad, bad
    finally:
        ops.set_deterministic(False)


def _store_view(store, flat, name):
    """The slice of a flat buffer (shaped like store.grad) that holds parameter ``name``."""
    v = store.grad_view(name)
    off = (v.data_ptr() - store.grad.data_ptr()) // v.element_size()
    return flat[off:off + v.numel()]


@pytest.mark.parametrize("B,T,nh,nkv,hd,pads", [
    (2, 64, 2, 2, 64, None), (2, 192, 4, 2, 64, None), (1, 1024, 4, 4, 64, None), (3, 512, 8, 2, 64, None),
    (2, 320, 4, 4, 32, None), (2, 256, 4, 4, 64, (0, 100)), (2, 1024, 16, 16, 64, (0, 700)),
])
@pytest.mark.parametrize("variant", ["d", "d8", "dx", "d8x", "r"])
def test_attention_fwd_variants(B, T, nh, nkv, hd, pads, variant, monkeypatch):
    """Forward kernels on pre-rotated q|k (the fused-RoPE path): the LDS-DMA kernel with 128- and
    256-query blocks ('d', 'd8'; 'x' = its cheaper-mask / split-sum variant) and the register-staged
    one ('r') against fp32 torch, output and log-sum-exp; T % 128 == 64 leaves idle waves in the last
    query block."""
    from nanodiloco_amd.ops import _ext
    from nanodiloco_amd.ops.attention import key_start
    monkeypatch.setenv("ND_ATTN_ABL", "32" if variant.endswith("x") else "0")  # x: the ILP softmax variant
    variant = variant.rstrip("x")
    monkeypatch.setenv("ND_ATTN_FWD", variant[0])
    monkeypatch.setenv("ND_ATTN_FWD_W", variant[1:] if variant[0] == "d" and variant[1:] else "4")
    ld = (nh + 2 * nkv) * hd
    qkv = torch.randn(B * T, ld, device=DEV).bfloat16()
    qkv[T // 2, nh * hd:(nh + 1) * hd] *= 20  # a late key with a large score: deferred-max rescale path
    k, v = qkv[:, nh * hd:], qkv[:, (nh + nkv) * hd:]
    ks = None
    if pads is not None:
        mask = torch.ones(B, T, dtype=torch.long, device=DEV)
        for b, p in enumerate(pads):
            mask[b, :p] = 0
        ks = key_start(mask)
    o = torch.empty(B * T, nh * hd, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, nh, T, device=DEV)
    L = _ext.lib()
    _ext.check(L.nd_attn_fwd_ks(qkv.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, nh, nkv, T,
                                hd, ld, nh * hd, 0, 0, hd ** -0.5, ks.data_ptr() if ks is not None else 0,
                                _ext.stream_ptr(qkv.device)), "fwd")
    q4, k4, v4 = ref.split_qkv(qkv.float(), B, T, nh, nkv, hd)
    rep = nh // nkv
    k4, v4 = k4.repeat_interleave(rep, 1), v4.repeat_interleave(rep, 1)
    s = (q4 @ k4.transpose(-1, -2)) * hd ** -0.5
    i = torch.arange(T, device=DEV)
    allowed = (i[None, :] <= i[:, None])[None, None].expand(B, 1, T, T).clone()
    if ks is not None:
        allowed &= (i[None, None, None, :] >= ks[:, None, None, None])
    s = s.masked_fill(~allowed, float("-inf"))
    lse_ref = torch.logsumexp(s, -1)  # natural log; the kernel stores log2 units
    p = torch.softmax(s, -1).nan_to_num(0.0)
    oref = (p @ v4).transpose(1, 2).reshape(B * T, nh * hd)
    assert torch.isfinite(o.float()).all()
    assert rel(o, oref) < 1e-2, rel(o, oref)
    valid = torch.isfinite(lse_ref)
    assert (lse[valid] / 1.4426950408889634 - lse_ref[valid]).abs().max().item() < 2e-2
    if ks is not None:
        pad_rows = ~allowed[:, 0].any(-1).reshape(-1)
        assert (o[pad_rows] == 0).all()


@pytest.mark.parametrize("B,T,nh,nkv,hd,pads", [
    (2, 64, 2, 2, 64, None), (2, 192, 4, 2, 64, None), (1, 1024, 4, 4, 64, None), (2, 320, 4, 4, 32, None),
    (2, 256, 4, 4, 64, (0, 100)), (2, 1024, 8, 2, 64, (0, 700)),
])
@pytest.mark.parametrize("variant", ["o", "o8", "k8"])
def test_attention_bwd_dq_variants(B, T, nh, nkv, hd, pads, variant, monkeypatch):
    """Fused backward (dQ kernel with the row statistics, then dK/dV) with 128- / 256-query dQ blocks
    ('o', 'o8') and 256-key dK/dV blocks ('k8'): all three gradients against fp32."""
    from nanodiloco_amd.ops.attention import key_start, rope_cache
    monkeypatch.setenv("ND_ATTN_DQ_W", variant[1:] if variant[0] == "o" and variant[1:] else "4")
    monkeypatch.setenv("ND_ATTN_DKDV_W", "8" if variant == "k8" else "4")  # 256-key dK/dV blocks
    ld = (nh + 2 * nkv) * hd
    ks = None
    if pads is not None:
        mask = torch.ones(B, T, dtype=torch.long, device=DEV)
        for b, p in enumerate(pads):
            mask[b, :p] = 0
        ks = key_start(mask)
    qkv = torch.randn(B * T, ld, device=DEV).bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, DEV)
    x = qkv.clone().requires_grad_(True)
    o = ops.attention(x, cos, sin, B, T, nh, nkv, hd, kstart=ks)
    xr = qkv.float().requires_grad_(True)
    orf = ref.attention_block(xr, cos, sin, B, T, nh, nkv, hd, kstart=ks)
    do = torch.randn_like(orf)
    o.backward(do.bfloat16())
    orf.backward(do.bfloat16().float())
    g, gr = x.grad.float(), xr.grad
    assert torch.isfinite(g).all()
    nq, nk = nh * hd, nkv * hd
    for name, sl in (("dq", slice(0, nq)), ("dk", slice(nq, nq + nk)), ("dv", slice(nq + nk, None))):
        assert rel(g[:, sl], gr[:, sl]) < 3e-2, (name, rel(g[:, sl], gr[:, sl]))


@pytest.mark.parametrize("B,T,nh,nkv,hd,pads", [
    (2, 192, 4, 2, 64, None), (1, 1024, 4, 4, 64, None), (2, 320, 4, 4, 32, None), (1, 256, 2, 2, 128, None),
    (2, 1024, 8, 2, 64, (0, 700)),
])
@pytest.mark.parametrize("nb", ["2", "3", "4"])
def test_attention_dkdv_prefetch_depth_bitwise(B, T, nh, nkv, hd, pads, nb, monkeypatch):
    """dK/dV with 64-query tiles and NB LDS buffers (ND_ATTN_DKDV_NB, profiles/r4_attention_dkdv_ablation.md):
    the same 32-query steps in the same order as the default kernel, so dQ / dK / dV are bitwise equal."""
    from nanodiloco_amd.ops.attention import key_start, rope_cache
    ld = (nh + 2 * nkv) * hd
    ks = None
    if pads is not None:
        mask = torch.ones(B, T, dtype=torch.long, device=DEV)
        for b, p in enumerate(pads):
            mask[b, :p] = 0
        ks = key_start(mask)
    qkv = torch.randn(B * T, ld, device=DEV).bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, DEV)
    do = torch.randn(B * T, nh * hd, device=DEV).bfloat16()

    def grads():
        x = qkv.clone().requires_grad_(True)
        ops.attention(x, cos, sin, B, T, nh, nkv, hd, kstart=ks).backward(do)
        return x.grad

    monkeypatch.delenv("ND_ATTN_DKDV_NB", raising=False)
    g0 = grads()
    monkeypatch.setenv("ND_ATTN_DKDV_NB", nb)
    g1 = grads()
    assert torch.isfinite(g0.float()).all()
    assert torch.equal(g0, g1)
