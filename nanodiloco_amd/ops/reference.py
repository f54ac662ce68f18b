"""Pure-PyTorch reference implementations of every hot op.

These are (a) the compute path on CPU (BASELINE config 1: CPU/gloo), (b) the fp32 numerics
oracle every HIP kernel is tested against, and (c) the explicit ``--ops torch`` baseline on GPU.
Semantics follow HF ``LlamaForCausalLM`` exactly (HF/models/llama/modeling_llama.py):

* RMSNorm upcasts to fp32, ``x * rsqrt(mean(x^2) + eps)``, casts back, then ``* w``  (:62-67)
* RoPE uses the half-split ``rotate_half`` convention, fp32 tables cast to the input dtype (:108-160)
* attention is causal SDPA with scale ``head_dim**-0.5`` and GQA by KV repetition (:226-281)
* SwiGLU MLP ``down(silu(gate(x)) * up(x))`` (:169-176)
* loss is mean token cross-entropy on fp32 logits over shifted labels, ignore_index=-100
  (HF/loss/loss_utils.py:32-71)
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- norms
def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    dt = x.dtype
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    y = xf * torch.rsqrt(var + eps)
    return w.to(dt) * y.to(dt) if w.dtype != torch.float32 else (w * y).to(dt)


def rmsnorm_hf(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    """Literal HF order of operations: ``weight * hidden.to(input_dtype)``."""
    dt = x.dtype
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return w * (xf * torch.rsqrt(var + eps)).to(dt)


def rmsnorm_backward(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, eps: float):
    """Returns (dx fp32, dw fp32) for y = w * x * rstd, all math in fp32."""
    xf, dyf, wf = x.float(), dy.float(), w.float()
    rstd = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    xhat = xf * rstd
    dw = (dyf * xhat).reshape(-1, x.shape[-1]).sum(0)
    g = dyf * wf
    dx = rstd * (g - xhat * (g * xhat).mean(-1, keepdim=True))
    return dx, dw


# ----------------------------------------------------------------------------- rope
def rope_inv_freq(head_dim: int, theta: float, scaling: Optional[dict] = None, device=None) -> torch.Tensor:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64, device=device).float() / head_dim))
    if scaling:
        kind = scaling.get("rope_type", scaling.get("type", "default"))
        if kind == "linear":
            inv = inv / float(scaling["factor"])
        elif kind == "llama3":
            factor = float(scaling["factor"])
            lo, hi = float(scaling["low_freq_factor"]), float(scaling["high_freq_factor"])
            old = float(scaling["original_max_position_embeddings"])
            lo_wl, hi_wl = old / lo, old / hi
            wl = 2 * math.pi / inv
            inv_l = torch.where(wl > lo_wl, inv / factor, inv)
            smooth = (old / wl - lo) / (hi - lo)
            smoothed = (1 - smooth) * inv_l / factor + smooth * inv_l
            is_med = ~(wl < hi_wl) & ~(wl > lo_wl)
            inv = torch.where(is_med, smoothed, inv_l)
    return inv


def rope_tables(seq_len: int, head_dim: int, theta: float, scaling: Optional[dict] = None,
                device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 cos/sin of shape [T, head_dim] (HF ``cat(freqs, freqs)`` layout)."""
    inv = rope_inv_freq(head_dim, theta, scaling, device=device)
    pos = torch.arange(seq_len, dtype=torch.float32, device=device)
    freqs = torch.outer(pos, inv)
    emb = torch.cat([freqs, freqs], dim=-1)
    return emb.cos(), emb.sin()


def rotate_half(x):
    h = x.shape[-1] // 2
    return torch.cat([-x[..., h:], x[..., :h]], dim=-1)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x: [B, H, T, hd]; cos/sin: [T, hd] fp32 (cast to x.dtype like HF)."""
    c, s = cos.to(x.dtype), sin.to(x.dtype)
    return x * c + rotate_half(x) * s


# ----------------------------------------------------------------------------- attention
def split_qkv(qkv: torch.Tensor, B: int, T: int, nh: int, nkv: int, hd: int):
    q, k, v = qkv.view(B, T, -1).split([nh * hd, nkv * hd, nkv * hd], dim=-1)
    q = q.reshape(B, T, nh, hd).transpose(1, 2)
    k = k.reshape(B, T, nkv, hd).transpose(1, 2)
    v = v.reshape(B, T, nkv, hd).transpose(1, 2)
    return q, k, v


def causal_attention(q, k, v, scale: Optional[float] = None):
    """q: [B, H, T, hd], k/v: [B, Hkv, T, hd] -> [B, H, T, hd].  Explicit math (no SDPA) for the oracle."""
    B, H, T, hd = q.shape
    rep = H // k.shape[1]
    if rep > 1:
        k = k.repeat_interleave(rep, dim=1)
        v = v.repeat_interleave(rep, dim=1)
    scale = hd ** -0.5 if scale is None else scale
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    mask = torch.ones(T, T, dtype=torch.bool, device=q.device).triu(1)
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.matmul(p, v.float()).to(q.dtype)


def padded_causal_mask(kstart: torch.Tensor, T: int) -> torch.Tensor:
    """Boolean [B, 1, T, T] (True = attend): causal & key is not a left pad (HF's sdpa mask).  Pad
    query rows are fully masked; torch SDPA returns 0 for them, as the attention kernels do."""
    t = torch.arange(T, device=kstart.device)
    causal = t[None, :] <= t[:, None]
    real_k = t.view(1, 1, T) >= kstart.view(-1, 1, 1).to(t.dtype)
    return (causal[None] & real_k).unsqueeze(1)


def attention_block(qkv: torch.Tensor, cos, sin, B: int, T: int, nh: int, nkv: int, hd: int,
                    use_sdpa: bool = True, kstart: torch.Tensor = None) -> torch.Tensor:
    """qkv [B*T, (nh+2nkv)*hd] -> RoPE -> causal attention -> [B*T, nh*hd] (autograd-capable).
    ``kstart``: left-padding key start per sequence (see ``ops.attention.key_start``)."""
    q, k, v = split_qkv(qkv, B, T, nh, nkv, hd)
    q = apply_rope(q, cos[:T], sin[:T])
    k = apply_rope(k, cos[:T], sin[:T])
    if kstart is not None:
        mask = padded_causal_mask(kstart.to(qkv.device), T)
        if nkv != nh:
            k = k.repeat_interleave(nh // nkv, dim=1)
            v = v.repeat_interleave(nh // nkv, dim=1)
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
        return o.transpose(1, 2).reshape(B * T, nh * hd)
    if use_sdpa:
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=(nkv != nh))
    else:
        o = causal_attention(q, k, v)
    return o.transpose(1, 2).reshape(B * T, nh * hd)


# ----------------------------------------------------------------------------- mlp
def swiglu(gate_up: torch.Tensor) -> torch.Tensor:
    g, u = gate_up.chunk(2, dim=-1)
    return F.silu(g) * u


def swiglu_backward(dy: torch.Tensor, gate_up: torch.Tensor) -> torch.Tensor:
    g, u = gate_up.float().chunk(2, dim=-1)
    dyf = dy.float()
    sg = torch.sigmoid(g)
    silu = g * sg
    dg = dyf * u * (sg * (1 + g * (1 - sg)))
    du = dyf * silu
    return torch.cat([dg, du], dim=-1).to(gate_up.dtype)


# ----------------------------------------------------------------------------- loss
def shift_labels(labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """HF ForCausalLMLoss shift: position t predicts labels[t+1]; last position ignored."""
    return F.pad(labels[:, 1:], (0, 1), value=ignore_index)


def cross_entropy_loss(logits: torch.Tensor, targets: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    return F.cross_entropy(logits.float().view(-1, logits.shape[-1]), targets.view(-1),
                           ignore_index=ignore_index, reduction="mean")
