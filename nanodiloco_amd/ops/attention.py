"""RoPE + causal flash attention on the packed QKV GEMM output (K4 + K6).

Input ``qkv`` is the fused q|k|v projection output ``[B*T, (nh + 2*nkv) * hd]`` (token-major, heads
packed).  The HIP path never transposes to ``[B, H, T, hd]``: the attention kernels take
(batch, head, token) strides and read 128-B head rows straight out of the packed buffer, and
write ``O`` as ``[B*T, nh*hd]`` -- exactly the o_proj GEMM input.

HIP path (RoPE: q|k rotated in place by one streaming pass -- no copy; dq/dk are un-rotated inside the
backward kernels' store epilogues, so the backward needs no extra pass)
  fwd: ``nd_rope_inplace`` then ``nd_attn_fwd``  -- MFMA flash attention, online softmax, saves LSE (fp32, log2 domain)
  bwd: ``nd_attn_bwd_fused`` = a query-parallel dQ kernel that also computes delta = rowsum(dO * O)
       and the dK/dV kernel's seeds, then a key-parallel dK/dV kernel (both recompute P from LSE; no
       atomics -> deterministic); ``nd_attn_bwd_pre`` + ``nd_attn_bwd`` is the unfused form.
``nd_rope_inplace`` (stand-alone rotation kernel) remains available for other callers.
GQA (nkv < nh) is handled by head-index mapping inside the kernels (no K/V repetition).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch

from . import _ext
from . import reference as ref

_TABLES: Dict[Tuple, Tuple[torch.Tensor, torch.Tensor]] = {}


def rope_cache(T: int, hd: int, theta: float, scaling, device) -> Tuple[torch.Tensor, torch.Tensor]:
    key = (T, hd, float(theta), repr(scaling), str(device))
    t = _TABLES.get(key)
    if t is None:
        cos, sin = ref.rope_tables(T, hd, theta, scaling, device="cpu")
        t = (cos.to(device).contiguous(), sin.to(device).contiguous())
        _TABLES[key] = t
    return t


def _rope(qkv, cos, sin, B, T, nh, nkv, hd, inverse):
    L = _ext.lib()
    _ext.check(L.nd_rope_inplace(_ext.ptr(qkv), _ext.dtcode(qkv), _ext.ptr(cos), _ext.ptr(sin), B * T, T,
                                 nh, nkv, hd, qkv.shape[1], 1 if inverse else 0, _ext.stream_ptr(qkv.device)),
               "nd_rope_inplace")


_FUSED_STATS = {"enabled": True}


def set_attn_fused_stats(enabled: bool) -> None:
    """Backward row statistics computed inside the dQ kernel (default) vs the separate
    delta / statistics kernels (A/B)."""
    _FUSED_STATS["enabled"] = bool(enabled)


class FlashAttnFn(torch.autograd.Function):
    """RoPE is applied to q|k IN PLACE in the packed projection output (one streaming pass, no copy):
    that buffer is this op's private input -- the projection's backward saved its input, not its
    output -- and it is saved here only after the rotation.  The backward kernels un-rotate dq/dk in
    their store epilogues (rope_mode 2), so the gradient returned is w.r.t. the raw projection."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, B, T, nh, nkv, hd, kstart=None, rotated=False):
        ld = qkv.shape[1]
        if not rotated:  # else the projection GEMM's epilogue already rotated q|k
            _rope(qkv, cos, sin, B, T, nh, nkv, hd, inverse=False)
        k = qkv[:, nh * hd:]
        v = qkv[:, (nh + nkv) * hd:]
        o = torch.empty(B * T, nh * hd, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(B, nh, T, dtype=torch.float32, device=qkv.device)
        L = _ext.lib()
        ks = _ext.ptr(kstart) if kstart is not None else 0
        _ext.check(L.nd_attn_fwd_ks(_ext.ptr(qkv), _ext.ptr(k), _ext.ptr(v), _ext.ptr(o), _ext.ptr(lse),
                                    B, nh, nkv, T, hd, ld, nh * hd, 0, 0, float(hd ** -0.5), ks,
                                    _ext.stream_ptr(qkv.device)), "nd_attn_fwd_ks")
        ctx.save_for_backward(qkv, o, lse, cos, sin)
        ctx.kstart = kstart
        ctx.dims = (B, T, nh, nkv, hd)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, cos, sin = ctx.saved_tensors
        B, T, nh, nkv, hd = ctx.dims
        do = do.contiguous()
        ld = qkv.shape[1]
        L = _ext.lib()
        dev = do.device
        ks = _ext.ptr(ctx.kstart) if ctx.kstart is not None else 0
        if _FUSED_STATS["enabled"] and T % 64 == 0:
            # dQ kernel computes delta = rowsum(dO * O) itself and seeds the dK/dV kernel
            dqkv = torch.empty_like(qkv)
            k, v = qkv[:, nh * hd:], qkv[:, (nh + nkv) * hd:]
            dk, dv = dqkv[:, nh * hd:], dqkv[:, (nh + nkv) * hd:]
            ws = torch.empty(2, B, nh, T, dtype=torch.float32, device=dev)
            _ext.check(L.nd_attn_bwd_fused_ks(_ext.ptr(qkv), _ext.ptr(k), _ext.ptr(v), _ext.ptr(o), _ext.ptr(do),
                                              _ext.ptr(lse), _ext.ptr(dqkv), _ext.ptr(dk), _ext.ptr(dv), _ext.ptr(ws),
                                              B, nh, nkv, T, hd, ld, nh * hd, _ext.ptr(cos), _ext.ptr(sin),
                                              float(hd ** -0.5), 2, ks, _ext.stream_ptr(dev)), "nd_attn_bwd_fused_ks")
            return dqkv, None, None, None, None, None, None, None, None, None
        delta = torch.empty(B, nh, T, dtype=torch.float32, device=dev)
        _ext.check(L.nd_attn_bwd_pre(_ext.ptr(o), _ext.ptr(do), _ext.ptr(delta), B, nh, T, hd, nh * hd,
                                     _ext.stream_ptr(dev)), "nd_attn_bwd_pre")
        dqkv = torch.empty_like(qkv)
        k, v = qkv[:, nh * hd:], qkv[:, (nh + nkv) * hd:]
        dk, dv = dqkv[:, nh * hd:], dqkv[:, (nh + nkv) * hd:]
        ws = torch.empty(2, B, nh, T, dtype=torch.float32, device=dev)  # -LSE/c, -delta for the dK/dV kernel
        _ext.check(L.nd_attn_bwd_ks(_ext.ptr(qkv), _ext.ptr(k), _ext.ptr(v), _ext.ptr(do), _ext.ptr(lse),
                                    _ext.ptr(delta), _ext.ptr(dqkv), _ext.ptr(dk), _ext.ptr(dv), _ext.ptr(ws),
                                    B, nh, nkv, T, hd, ld, nh * hd, _ext.ptr(cos), _ext.ptr(sin), float(hd ** -0.5), 2,
                                    ks, _ext.stream_ptr(dev)), "nd_attn_bwd_ks")
        return dqkv, None, None, None, None, None, None, None, None, None


def key_start(attention_mask: torch.Tensor) -> torch.Tensor:
    """Per-sequence first real key (int32 [B]) of an HF ``attention_mask`` [B, T] (1 = token, 0 = pad).

    Left padding ([0..0, 1..1]) gives the pad count; right padding ([1..1, 0..0]) gives 0 -- causal
    attention already keeps every real query off the trailing pad keys.  Masks with holes (a pad
    between real tokens) are not expressible as a key start: ``check_padding`` rejects them."""
    m = attention_mask.to(torch.int32)
    return (m.cumsum(1) == 0).sum(1).to(torch.int32)


def check_padding(attention_mask: torch.Tensor) -> None:
    """Raise unless every row is left- or right-padded (one contiguous run of real tokens)."""
    m = attention_mask.to(torch.int32)
    transitions = (m[:, 1:] != m[:, :-1]).sum(1)
    if bool((transitions > 2).any()) or bool(((transitions == 2) & (m[:, 0] == 1)).any()):
        raise ValueError("attention_mask rows must be one contiguous run of tokens (left or right padding)")


def attention(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, B: int, T: int, nh: int, nkv: int,
              hd: int, inplace: bool = False, kstart: torch.Tensor = None, rotated: bool = False) -> torch.Tensor:
    """Causal self-attention with RoPE; qkv [B*T, (nh+2nkv)*hd] -> [B*T, nh*hd].

    ``kstart`` (int32 [B], from :func:`key_start`) masks left padding: real queries (t >= kstart[b])
    never see the pad keys t' < kstart[b] -- the reference's causal + padding mask
    (REF/nanodiloco/main.py:79-88,109 -> HF SDPA).  ``inplace=True`` lets the HIP path rotate q|k
    inside ``qkv`` itself (the model passes it for the projection output it owns); otherwise a private
    copy is rotated.  ``rotated=True``: q|k already carry RoPE (the projection GEMM's epilogue,
    ops/linear.py LinearRopeFn); the backward still returns the gradient w.r.t. the un-rotated q|k."""
    if rotated and not qkv.is_cuda:
        raise ValueError("rotated=True is a GPU-path contract (fused RoPE GEMM epilogue)")
    if _ext.use_hip(qkv):
        x = qkv.contiguous()
        if not inplace and x.data_ptr() == qkv.data_ptr():
            x = x.clone()  # never rotate a caller-visible tensor
        ks = kstart.to(device=qkv.device, dtype=torch.int32).contiguous() if kstart is not None else None
        return FlashAttnFn.apply(x, cos, sin, B, T, nh, nkv, hd, ks, bool(rotated))
    return ref.attention_block(qkv, cos, sin, B, T, nh, nkv, hd, use_sdpa=True, kstart=kstart)
