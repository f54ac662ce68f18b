"""T2: our Llama (PyTorch path) vs HF LlamaForCausalLM with the same weights (fp32)."""
import pytest
import torch

from nanodiloco_amd.config import LlamaConfig
from nanodiloco_amd.models import LlamaForCausalLM, ParamStore

transformers = pytest.importorskip("transformers")


@pytest.mark.parametrize("cfgd", [
    dict(hidden_size=64, intermediate_size=128, num_attention_heads=4, num_hidden_layers=2, vocab_size=97),
    dict(hidden_size=64, intermediate_size=96, num_attention_heads=4, num_key_value_heads=2, num_hidden_layers=2,
         vocab_size=101, rms_norm_eps=1e-5),
    dict(hidden_size=32, intermediate_size=64, num_attention_heads=2, num_hidden_layers=1, vocab_size=64,
         tie_word_embeddings=True),
])
def test_logits_loss_grads_match_hf(cfgd):
    torch.manual_seed(0)
    c = LlamaConfig.from_dict(cfgd)
    m = LlamaForCausalLM(c).init_weights(1)
    hf = transformers.LlamaForCausalLM(transformers.LlamaConfig(**cfgd, attn_implementation="eager")).float()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    hf.load_state_dict(sd, strict=False)
    if c.tie_word_embeddings:
        hf.tie_weights()
    ids = torch.randint(0, c.vocab_size, (3, 24))
    labels = ids.clone()
    labels[0, :5] = -100
    out = m(ids, labels=labels)
    out.loss.backward()
    ho = hf(input_ids=ids, labels=labels)
    ho.loss.backward()
    assert abs(out.loss.item() - ho.loss.item()) < 1e-5
    for n, p in hf.named_parameters():
        assert torch.allclose(p.grad, m.store.grad_view(n), atol=2e-6, rtol=1e-4), n
    logits = m(ids).logits
    assert torch.allclose(logits, ho.logits, atol=1e-5)


def test_loss_scale_scales_grads_only():
    c = LlamaConfig.from_dict(dict(hidden_size=32, intermediate_size=64, num_attention_heads=2,
                                   num_hidden_layers=1, vocab_size=50))
    m = LlamaForCausalLM(c).init_weights(0)
    ids = torch.randint(0, 50, (2, 16))
    l1 = m(ids, labels=ids).loss
    l1.backward()
    g1 = m.store.grad.clone()
    m.store.zero_grad()
    l2 = m(ids, labels=ids, loss_scale=0.25).loss
    l2.backward()
    assert torch.allclose(l1, l2)
    assert torch.allclose(m.store.grad, 0.25 * g1, atol=1e-7)


def test_param_store_layout():
    c = LlamaConfig.from_dict(dict(hidden_size=64, intermediate_size=128, num_attention_heads=4,
                                   num_key_value_heads=2, num_hidden_layers=2, vocab_size=100))
    m = LlamaForCausalLM(c)
    st = m.store
    assert st.numel % (64 * 840) == 0
    for n in st.names:
        assert st.offsets[n] % 64 == 0 or "k_proj" in n or "v_proj" in n or "up_proj" in n
    qkv = st.fused_view("master", ["model.layers.0.self_attn.q_proj.weight", "model.layers.0.self_attn.k_proj.weight",
                                   "model.layers.0.self_attn.v_proj.weight"])
    assert qkv.shape == (64 + 32 + 32, 64)
    st.master_view("model.layers.0.self_attn.k_proj.weight").fill_(3.0)
    assert (qkv[64:96] == 3.0).all()
    assert list(m.state_dict().keys()) == [n for n, _ in c.param_shapes()]


def test_activation_checkpointing_same_grads():
    c = LlamaConfig.from_dict(dict(hidden_size=32, intermediate_size=64, num_attention_heads=2,
                                   num_hidden_layers=2, vocab_size=50))
    ids = torch.randint(0, 50, (2, 16))
    m1 = LlamaForCausalLM(c).init_weights(0)
    m1(ids, labels=ids).loss.backward()
    m2 = LlamaForCausalLM(c, activation_checkpointing=True).init_weights(0)
    m2(ids, labels=ids).loss.backward()
    assert torch.allclose(m1.store.grad, m2.store.grad, atol=1e-7)


def test_rmsnorm_res_fuses_residual_grad():
    """ops.rmsnorm_res(x) == (rmsnorm(x), x) with the residual gradient summed inside the node."""
    from nanodiloco_amd import ops
    torch.manual_seed(0)
    x = torch.randn(6, 32, dtype=torch.float64)
    w = torch.randn(32, dtype=torch.float64)
    up = torch.randn(6, 32, dtype=torch.float64)
    ur = torch.randn(6, 32, dtype=torch.float64)
    outs = []
    for fused in (True, False):
        xx = x.clone().requires_grad_(True)
        gw = torch.zeros_like(w)
        if fused:
            y, h = ops.rmsnorm_res(xx, w, gw, 1e-5)
        else:
            y, h = ops.rmsnorm(xx, w, gw, 1e-5), xx
        ((y * up).sum() + (h * ur).sum()).backward()
        outs.append((y.detach(), xx.grad, gw))
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b)
    # residual output unused: the gradient is the norm's alone
    xx = x.clone().requires_grad_(True)
    y, _ = ops.rmsnorm_res(xx, w, None, 1e-5)
    (y * up).sum().backward()
    xr = x.clone().requires_grad_(True)
    (ops.rmsnorm(xr, w, None, 1e-5) * up).sum().backward()
    torch.testing.assert_close(xx.grad, xr.grad)


def test_bf16_residual_stream_tracks_fp32():
    """--residual-dtype bf16 on the PyTorch path: the residual stream and its gradient are bf16 tensors, and loss /
    gradients stay within bf16 rounding of the fp32-residual model (same weights, same batch)."""
    c = LlamaConfig.from_dict(dict(hidden_size=64, intermediate_size=128, num_attention_heads=4,
                                   num_key_value_heads=2, num_hidden_layers=2, vocab_size=97))
    ids = torch.randint(0, 97, (3, 24), generator=torch.Generator().manual_seed(0))
    res = {}
    for rdt in (None, torch.bfloat16):
        m = LlamaForCausalLM(c, residual_dtype=rdt).init_weights(1)
        loss = m(ids, labels=ids).loss
        loss.backward()
        res[rdt] = (loss.item(), m.store.grad.clone())
    (l32, g32), (l16, g16) = res[None], res[torch.bfloat16]
    assert abs(l32 - l16) < 1e-2 * l32
    assert ((g32 - g16).norm() / g32.norm()).item() < 3e-2
    with pytest.raises(ValueError):
        LlamaForCausalLM(c, residual_dtype=torch.float16)


def test_bf16_residual_add_rmsnorm_rounds_h_new():
    """The PyTorch fallback of add_rmsnorm on a bf16 residual: h_new is the RNE-rounded sum and the norm's
    statistics are those of the rounded value (what the HIP kernel stores and the backward recomputes from)."""
    from nanodiloco_amd import ops
    torch.manual_seed(0)
    h = torch.randn(5, 32).bfloat16()
    a = torch.randn(5, 32).bfloat16()
    w = torch.randn(32)
    y, hn = ops.add_rmsnorm(h, a, w, None, 1e-5, torch.float32)
    assert hn.dtype == torch.bfloat16 and torch.equal(hn, (h.float() + a.float()).bfloat16())
    x = hn.float()
    torch.testing.assert_close(y, w * (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5)))


@pytest.mark.parametrize("side", ["left", "right"])
def test_padded_batch_matches_hf_attention_mask(side):
    """Padded batches (the reference's tokenizer.pad + attention_mask, REF/nanodiloco/main.py:79-88,109):
    loss, grads and the logits of every real token match HF given the same attention_mask."""
    torch.manual_seed(0)
    cfgd = dict(hidden_size=64, intermediate_size=96, num_attention_heads=4, num_key_value_heads=2,
                num_hidden_layers=2, vocab_size=101, rms_norm_eps=1e-5)
    c = LlamaConfig.from_dict(cfgd)
    m = LlamaForCausalLM(c).init_weights(3)
    # the reference builds LlamaForCausalLM with the default (sdpa) attention: fully masked (left-pad)
    # query rows come out as 0, which decides the prediction made at the last pad position
    hf = transformers.LlamaForCausalLM(transformers.LlamaConfig(**cfgd, attn_implementation="sdpa")).float()
    hf.load_state_dict({k: v.clone() for k, v in m.state_dict().items()}, strict=False)
    B, T = 3, 20
    ids = torch.randint(0, c.vocab_size, (B, T))
    mask = torch.ones(B, T, dtype=torch.long)
    for b, npad in enumerate([0, 5, 11]):
        if npad:
            if side == "left":
                mask[b, :npad] = 0
            else:
                mask[b, T - npad:] = 0
    ids[mask == 0] = 2  # pad token
    labels = ids.clone()
    labels[mask == 0] = -100
    out = m(ids, labels=labels, attention_mask=mask)
    out.loss.backward()
    ho = hf(input_ids=ids, attention_mask=mask, labels=labels)
    ho.loss.backward()
    assert abs(out.loss.item() - ho.loss.item()) < 1e-5, (out.loss.item(), ho.loss.item())
    for n, p in hf.named_parameters():
        assert torch.allclose(p.grad, m.store.grad_view(n), atol=2e-6, rtol=1e-4), n
    logits = m(ids, attention_mask=mask).logits
    # left: every position matches (pad rows attend to nothing on both sides); right: trailing pad
    # queries still see the real keys in HF (and everything causal here) -- they carry no loss
    sel = torch.ones_like(mask, dtype=torch.bool) if side == "left" else mask.bool()
    assert torch.allclose(logits[sel], ho.logits[sel], atol=1e-5)


def test_key_start_and_padding_check():
    from nanodiloco_amd.ops import check_padding, key_start
    mask = torch.tensor([[0, 0, 1, 1], [1, 1, 1, 0], [1, 1, 1, 1], [0, 1, 1, 1]])
    assert key_start(mask).tolist() == [2, 0, 0, 1]
    check_padding(mask)
    with pytest.raises(ValueError):
        check_padding(torch.tensor([[1, 0, 1, 1]]))
