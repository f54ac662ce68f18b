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


@pytest.mark.parametrize("shape", [(1024, 2688), (96, 72)])
def test_fp8_weight_current_scaling(shape):
    """Fp8Weight: amax-only pass + one cast/transpose pass == torch current scaling of W and W^T."""
    w = (torch.randn(*shape, device="cuda") * 0.02).bfloat16()
    wq = fp8.Fp8Weight().get(w, version=0)
    s = fp8.FMAX[fp8.E4M3] / w.float().abs().max()
    ref = (w.float() * s).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert torch.allclose(wq.inv, (1.0 / s).reshape(1))
    assert torch.equal(wq.w8.view(torch.uint8), ref.view(torch.uint8))
    assert torch.equal(wq.wT8.view(torch.uint8), ref.t().contiguous().view(torch.uint8))
    assert wq.get(w, version=0) is wq and wq.version == 0


@pytest.fixture(params=["auto", "pp", "hipblaslt"])
def fp8_gemm(request):
    """The fp8 GEMM backends: the own ping-pong kernel (default; with the fused RoPE / SwiGLU epilogues
    in the model), and hipBLASLt (A/B)."""
    old = fp8.fp8_gemm_backend()
    fp8.set_fp8_gemm(request.param)
    yield request.param
    fp8.set_fp8_gemm(old)


@pytest.mark.parametrize("wgrad_fp8", [True, False])
def test_fp8_linear_close_to_fp32(wgrad_fp8, fp8_gemm):
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


@pytest.mark.parametrize("wgrad_fp8", [False, True], ids=["wgrad-bf16", "wgrad-fp8"])
def test_fp8_training_tracks_bf16(fp8_gemm, wgrad_fp8):
    cfg = LlamaConfig.from_dict(dict(hidden_size=256, intermediate_size=768, num_attention_heads=4,
                                     num_key_value_heads=4, num_hidden_layers=2, vocab_size=512))
    ids = torch.randint(0, 512, (8, 256), device="cuda")
    losses = {}
    for use_fp8 in (False, True):
        m = LlamaForCausalLM(cfg, "cuda", torch.bfloat16, fp8=use_fp8, fp8_wgrad=wgrad_fp8).init_weights(5)
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


@pytest.mark.parametrize("keep", ["rope", "mlp", "both"])
def test_fp8_keep_fused_tracks_bf16(keep):
    """--fp8-keep-fused: the kept projections run on the bf16 fused-epilogue GEMMs (no fp8 slot is
    created for them), the rest in fp8; the model still trains like the bf16 one."""
    cfg = LlamaConfig.from_dict(dict(hidden_size=256, intermediate_size=768, num_attention_heads=4,
                                     num_key_value_heads=4, num_hidden_layers=2, vocab_size=512))
    ids = torch.randint(0, 512, (8, 256), device="cuda")
    losses = {}
    try:
        for mode in ("bf16", keep):
            fp8.set_fp8_keep_fused("none" if mode == "bf16" else keep)
            m = LlamaForCausalLM(cfg, "cuda", torch.bfloat16, fp8=mode != "bf16").init_weights(5)
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
            losses[mode] = ls
            if m.fp8 is not None:
                kinds = {k.split(".")[1] for k in m.fp8.slots}
                assert "o" in kinds
                assert ("qkv" in kinds) == (keep == "mlp")
                assert ("gu" in kinds) == ("down" in kinds) == (keep == "rope")
    finally:
        fp8.set_fp8_keep_fused("none")
    b, f = losses["bf16"], losses[keep]
    assert f[-1] < 0.5 * f[0], f
    assert abs(f[-1] - b[-1]) < 0.15 * b[0], (b[-1], f[-1])


# ----------------------------------------------------------------- fused producer-side quantisation
def _target(fmt, scale=23.0):
    r = fp8.Fp8Recipe("cuda", capacity=4)
    k = r.new_slot(fmt)
    r.scale[k] = scale
    r.ready[k] = True
    return r, k, r.target(k, fmt)


@pytest.mark.parametrize("fmt", [fp8.E4M3, fp8.E5M2])
def test_fused_swiglu_quant_bitwise(fmt):
    """SwiGLU fwd/bwd fp8 side outputs == a separate cast of the bf16 outputs (bytes and amax)."""
    from nanodiloco_amd.ops.swiglu import SwiGLUFn
    gu = torch.randn(300, 2 * 2688, device="cuda").bfloat16().requires_grad_(True)
    r, k, q = _target(fmt)
    rb, kb, qb = _target(fp8.E5M2, 3.0)
    out = SwiGLUFn.apply(gu, q, qb)
    ref = fp8.cast(out.detach(), r.scale[k:k + 1], fmt)
    assert torch.equal(q.out.view(torch.uint8), ref.view(torch.uint8))
    assert r.amax[k].max().item() == out.detach().float().abs().max().item()
    dy = torch.randn_like(out)
    (dgu,) = torch.autograd.grad(out, gu, dy)
    q8 = rb.take_stashed(kb, dgu)
    assert q8 is not None
    refb = fp8.cast(dgu, rb.scale[kb:kb + 1], fp8.E5M2)
    assert torch.equal(q8.view(torch.uint8), refb.view(torch.uint8))
    assert rb.amax[kb].max().item() == dgu.float().abs().max().item()


@pytest.mark.parametrize("V", [32000, 16384])
def test_ce_fused_fp8_dlogits_bitwise(V):
    """nd_ce_fwd_bwd_q8 (the CE kernel writing the dlogits only as e5m2) == the bf16 CE kernel + a separate
    cast: fp8 bytes and amax bitwise, loss within float-atomic order; the logits buffer is left untouched."""
    from nanodiloco_amd.ops import _ext
    n = 1000
    logits = (3 * torch.randn(n, V, device="cuda")).bfloat16()
    tgt = torch.randint(0, V, (n,), device="cuda")
    tgt[::9] = -100
    scale = torch.tensor([1.0 / 800], device="cuda")
    L = _ext.lib()
    # reference: bf16 dlogits in place, then the separate cast
    ref_l = logits.clone()
    loss_ref = torch.zeros(1, device="cuda")
    _ext.check(L.nd_ce_fwd_bwd(ref_l.data_ptr(), _ext.dtcode(ref_l), tgt.data_ptr(), loss_ref.data_ptr(),
                               scale.data_ptr(), n, V, -100, 0, 0, 0.0, _ext.stream_ptr()), "ce")
    r, k, t = _target(fp8.E5M2, 2000.0)
    ref8 = fp8.cast(ref_l, r.scale[k:k + 1], fp8.E5M2)
    # fused
    r2, k2, t2 = _target(fp8.E5M2, 2000.0)
    q8 = t2.alloc((n, V), "cuda")
    fl = logits.clone()
    loss = torch.zeros(1, device="cuda")
    _ext.check(L.nd_ce_fwd_bwd_q8(fl.data_ptr(), _ext.dtcode(fl), tgt.data_ptr(), loss.data_ptr(), scale.data_ptr(),
                                  n, V, -100, 0, 0, *t2.args(q8), _ext.stream_ptr()), "ce_q8")
    torch.cuda.synchronize()
    assert torch.equal(fl, logits)
    assert torch.equal(q8.view(torch.uint8), ref8.view(torch.uint8))
    assert r2.amax[k2].max().item() == ref_l.float().abs().max().item()
    assert abs(loss.item() - loss_ref.item()) <= 1e-5 * abs(loss_ref.item())


def test_ce_fused_fp8_refuses_other_shapes():
    """Shapes outside the packed kernel's range come back as hipErrorInvalidValue (the caller casts separately)."""
    from nanodiloco_amd.ops import _ext
    n, V = 8, 1000
    logits = torch.randn(n, V, device="cuda").bfloat16()
    tgt = torch.randint(0, V, (n,), device="cuda")
    r, k, t = _target(fp8.E5M2)
    q8 = t.alloc((n, V), "cuda")
    loss, scale = torch.zeros(1, device="cuda"), torch.ones(1, device="cuda")
    rc = _ext.lib().nd_ce_fwd_bwd_q8(logits.data_ptr(), _ext.dtcode(logits), tgt.data_ptr(), loss.data_ptr(),
                                     scale.data_ptr(), n, V, -100, 0, 0, *t.args(q8), _ext.stream_ptr())
    assert rc == 1


@pytest.mark.parametrize("hdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("residual", [False, True])
def test_fused_rmsnorm_quant_bitwise(residual, hdt):
    """RMSNorm fwd (y -> e4m3) and bwd (branch grad -> e5m2) fp8 side outputs == separate casts (fp32 and bf16
    residual streams)."""
    rows, cols = 777, 1024
    h = torch.randn(rows, cols, device="cuda").to(hdt)
    a = torch.randn(rows, cols, device="cuda").bfloat16()
    w = 1 + 0.1 * torch.randn(cols, device="cuda")
    r, k, q = _target(fp8.E4M3, 50.0)
    rb, kb, qb = _target(fp8.E5M2, 1000.0)
    hr = h.clone().requires_grad_(True)
    ar = a.clone().requires_grad_(True)
    if residual:
        y, hn = ops.add_rmsnorm(hr, ar, w, None, 1e-5, torch.bfloat16, q8=q, q8_bwd=qb)
    else:
        y = ops.rmsnorm(hr, w, None, 1e-5, torch.bfloat16, q8=q)
    ref = fp8.cast(y.detach(), r.scale[k:k + 1], fp8.E4M3)
    assert torch.equal(q.out.view(torch.uint8), ref.view(torch.uint8))
    assert r.amax[k].max().item() == y.detach().float().abs().max().item()
    if residual:
        dy = torch.randn_like(y)
        (da,) = torch.autograd.grad(y, ar, dy)
        q8 = rb.take_stashed(kb, da)
        assert q8 is not None
        refb = fp8.cast(da, rb.scale[kb:kb + 1], fp8.E5M2)
        assert torch.equal(q8.view(torch.uint8), refb.view(torch.uint8))


def test_fused_quant_training_matches_separate_casts():
    """The fp8 model trains identically with producer-fused and with separate operand casts."""
    cfg = LlamaConfig.from_dict(dict(hidden_size=256, intermediate_size=512, num_attention_heads=4,
                                     num_hidden_layers=2, vocab_size=1000))
    batches = [torch.randint(0, 1000, (4, 256), device="cuda") for _ in range(6)]

    def run(fused):
        fp8.set_fused_quant(fused)
        try:
            m = LlamaForCausalLM(cfg, "cuda", torch.bfloat16, fp8=True).init_weights(2)
            opt = FlatAdamW(m.store, lr=1e-3)
            losses = []
            for i, ids in enumerate(batches):
                out = m(ids, labels=ids, loss_scale=0.5)
                out.loss.backward()
                losses.append(out.loss.detach())
                if i % 2 == 1:
                    opt.step()
                    opt.zero_grad()
                    m.fp8.recipe.update()
            torch.cuda.synchronize()
            return torch.stack(losses).cpu(), m.store.master.clone()
        finally:
            fp8.set_fused_quant(True)

    l0, p0 = run(False)
    l1, p1 = run(True)
    assert (l1 - l0).abs().max().item() < 2e-3, (l0, l1)
    assert ((p1 - p0).norm() / p0.norm()).item() < 1e-3


def test_fp8_fused_epilogues_track_unfused():
    """fp8 projections with RoPE / SwiGLU fused into the own fp8 GEMMs (default) train like the same fp8
    model with separate RoPE / SwiGLU passes, and actually take the fused path."""
    cfg = LlamaConfig.from_dict(dict(hidden_size=256, intermediate_size=768, num_attention_heads=4,
                                     num_key_value_heads=4, num_hidden_layers=2, vocab_size=512))
    ids = torch.randint(0, 512, (8, 256), device="cuda")
    losses = {}
    try:
        for fused in (False, True):
            fp8.set_fp8_fused_epilogues(fused)
            m = LlamaForCausalLM(cfg, "cuda", torch.bfloat16, fp8=True).init_weights(5)
            calls = {"rope": 0, "mlp": 0}
            orig_rope, orig_mlp = fp8.Fp8RopeFn.apply, fp8.Fp8MLPFn.apply

            def rope_apply(*a, _o=orig_rope):
                calls["rope"] += 1
                return _o(*a)

            def mlp_apply(*a, _o=orig_mlp):
                calls["mlp"] += 1
                return _o(*a)

            fp8.Fp8RopeFn.apply, fp8.Fp8MLPFn.apply = rope_apply, mlp_apply
            try:
                opt = FlatAdamW(m.store, lr=3e-3)
                ls = []
                for _ in range(20):
                    out = m(ids, labels=ids)
                    out.loss.backward()
                    opt.step()
                    m.fp8.recipe.update()
                    m.store.zero_grad()
                    ls.append(out.loss.item())
            finally:
                fp8.Fp8RopeFn.apply, fp8.Fp8MLPFn.apply = orig_rope, orig_mlp
            assert (calls["rope"] > 0) == fused and (calls["mlp"] > 0) == fused, calls
            losses[fused] = ls
    finally:
        fp8.set_fp8_fused_epilogues(True)
    u, f = losses[False], losses[True]
    assert f[-1] < 0.5 * f[0], f
    assert abs(f[-1] - u[-1]) < 0.1 * u[0], (u[-1], f[-1])


def test_fp8_lm_head_tracks_bf16_one_step():
    """The fp8 lm head (e4m3 logits GEMM, e5m2 dlogits into the fp8 dgrad / wgrad kernels, ops/cross_entropy.py)
    against the bf16 one on the same weights: loss, input gradient and weight gradient within fp8 tolerance."""
    from nanodiloco_amd.ops.cross_entropy import lm_head_ce
    torch.manual_seed(0)
    n, d, V = 1024, 256, 1024
    y = (torch.randn(n, d, device="cuda") * 0.5).bfloat16().requires_grad_(True)
    w = (torch.randn(V, d, device="cuda") * 0.05).bfloat16()
    t = torch.randint(0, V, (n,), device="cuda")
    res = {}
    for use in (False, True):
        gw = torch.zeros(V, d, device="cuda")
        f8 = (fp8.Fp8Linears("cuda", wgrad_fp8=True), 0, None) if use else None
        yy = y.detach().clone().requires_grad_(True)
        loss = lm_head_ce(yy, w, gw, t, 1.0, f8=f8)
        loss.backward()
        from nanodiloco_amd.ops.linear import join_wgrad
        join_wgrad()
        torch.cuda.synchronize()
        res[use] = (loss.item(), yy.grad.float(), gw)
    (lb, gb, wb), (lf, gf, wf) = res[False], res[True]
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    assert abs(lf - lb) < 0.01 * lb, (lf, lb)
    assert rel(gf, gb) < 0.15 and rel(wf, wb) < 0.15, (rel(gf, gb), rel(wf, wb))


def test_fp8_lm_head_fused_dlogits_match_separate_cast():
    """V = 32000 (the packed CE kernel's range): from the second call on (the slot has a scale), the CE kernel
    writes the e5m2 dlogits itself; loss, input gradient and weight gradient are bitwise those of the separate
    cast path (fused quantisation off), and so is the slot's amax."""
    from nanodiloco_amd.ops.cross_entropy import LM_KEY, lm_head_ce
    from nanodiloco_amd.ops.linear import join_wgrad
    torch.manual_seed(0)
    n, d, V = 512, 256, 32000
    y = (torch.randn(n, d, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(V, d, device="cuda") * 0.05).bfloat16()
    t = torch.randint(0, V, (n,), device="cuda")
    t[::11] = -100
    outs = []
    for fused in (True, False):
        fp8.set_fused_quant(fused)
        try:
            lin = fp8.Fp8Linears("cuda", wgrad_fp8=True)
            for _ in range(2):
                gw = torch.zeros(V, d, device="cuda")
                yy = y.clone().requires_grad_(True)
                loss = lm_head_ce(yy, w, gw, t, 1.0, f8=(lin, 0, None))
                loss.backward()
                join_wgrad()
            torch.cuda.synchronize()
            kdy = lin._slots(LM_KEY)[1]
            outs.append((loss.item(), yy.grad.clone(), gw.clone(), lin.recipe.amax[kdy].max().item()))
        finally:
            fp8.set_fused_quant(True)
    (l1, g1, w1, a1), (l2, g2, w2, a2) = outs
    assert abs(l1 - l2) <= 1e-5 * abs(l2)
    assert torch.equal(g1, g2) and torch.equal(w1, w2) and a1 == a2


def _fp8_model_steps(cfg, ids, steps, overlap=None, fused=None):
    """A few fp8 training steps (fp8 weight gradients); returns (per-step flat grads, final master weights)."""
    prev_ov = ops.wgrad_overlap_enabled()
    try:
        if overlap is not None:
            ops.set_wgrad_overlap(overlap)
        if fused is not None:
            fp8.set_fp8_fused_epilogues(fused)
        m = LlamaForCausalLM(cfg, "cuda", torch.bfloat16, fp8=True, fp8_wgrad=True).init_weights(11)
        opt = FlatAdamW(m.store, lr=2e-3)
        grads = []
        for _ in range(steps):
            out = m(ids, labels=ids)
            out.loss.backward()
            ops.join_wgrad()
            grads.append(m.store.grad.clone())
            opt.step()
            m.fp8.recipe.update()
            m.store.zero_grad()
        torch.cuda.synchronize()
        return grads, m.store.master.clone(), m
    finally:
        ops.set_wgrad_overlap(prev_ov)
        fp8.set_fp8_fused_epilogues(True)


def test_fp8_wgrad_side_stream_matches_serial():
    """fp8 weight gradients on the side stream (the trainer default: fp8_wgrad + wgrad_overlap) against the
    serial schedule: the same own kernels, so gradients and weights are bitwise equal (advisor r4)."""
    cfg = LlamaConfig.from_dict(dict(hidden_size=256, intermediate_size=768, num_attention_heads=4,
                                     num_key_value_heads=4, num_hidden_layers=2, vocab_size=512))
    ids = torch.randint(0, 512, (8, 256), device="cuda")
    ops.set_deterministic(True)
    try:
        g0, p0, _ = _fp8_model_steps(cfg, ids, 3, overlap=0)
        g1, p1, m = _fp8_model_steps(cfg, ids, 3, overlap=1)
    finally:
        ops.set_deterministic(False)
    for a, b in zip(g0, g1):
        assert torch.equal(a, b)
    assert torch.equal(p0, p1)


def test_fp8_fused_epilogue_gradients_match_unfused_one_step():
    """One step, same weights: the fused RoPE / SwiGLU / SwiGLU-backward fp8 GEMMs give parameter gradients as
    close to the bf16 model's as the unfused fp8 path does (per tensor, within 1.5x of its deviation) -- a wrong
    RoPE or SwiGLU backward (e.g. a gradient that is never un-rotated) lands O(1) away (advisor r4)."""
    cfg = LlamaConfig.from_dict(dict(hidden_size=256, intermediate_size=768, num_attention_heads=4,
                                     num_key_value_heads=4, num_hidden_layers=2, vocab_size=512))
    ids = torch.randint(0, 512, (8, 256), device="cuda")
    gu, _, mu = _fp8_model_steps(cfg, ids, 1, overlap=0, fused=False)
    gf, _, mf = _fp8_model_steps(cfg, ids, 1, overlap=0, fused=True)
    mb = LlamaForCausalLM(cfg, "cuda", torch.bfloat16).init_weights(11)
    mb(ids, labels=ids).loss.backward()
    ops.join_wgrad()
    torch.cuda.synchronize()
    gb = mb.store.grad
    rel = lambda x, y: ((x - y).norm() / y.norm().clamp_min(1e-20)).item()  # noqa: E731
    rows = []
    for name in mb.store.names:
        if "norm" in name:
            continue
        f, u, b = mf.store._view(gf[0], name), mu.store._view(gu[0], name), mb.store._view(gb, name)
        rows.append((name, rel(f, b), rel(u, b), rel(f, u)))
    print("\n".join(f"{n:45s} fused~bf16 {x:.3f} unfused~bf16 {y:.3f} fused~unfused {z:.3f}" for n, x, y, z in rows))
    for n, x, y, z in rows:
        assert x < 1.5 * y + 0.02 and x < 0.5, (n, x, y, z)
