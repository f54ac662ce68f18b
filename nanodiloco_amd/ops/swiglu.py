"""SwiGLU activation on the fused gate|up GEMM output (K7).

``act = silu(gu[:, :F]) * gu[:, F:]``.  HIP path: one memory-bound kernel each way with 16-B
vector loads (``nd_swiglu_fwd`` / ``nd_swiglu_bwd``); the backward writes the fused
d(gate|up) tensor that feeds the single fused dgrad/wgrad GEMM.
"""
from __future__ import annotations

import torch

from . import _ext
from . import reference as ref


class SwiGLUFn(torch.autograd.Function):
    """``q8`` / ``q8_bwd`` (fp8 inner step, ops/fp8.QuantTarget): the same kernels also write the e4m3
    copy of the activation (down-projection input) / the e5m2 copy of d(gate|up)."""

    @staticmethod
    def forward(ctx, gu, q8=None, q8_bwd=None):
        gu = gu.contiguous()
        n, f2 = gu.shape
        out = torch.empty(n, f2 // 2, dtype=gu.dtype, device=gu.device)
        if q8 is not None and gu.dtype == torch.bfloat16:
            q = q8.alloc((n, f2 // 2), gu.device)
            _ext.check(_ext.lib().nd_swiglu_fwd_q(_ext.ptr(gu), _ext.ptr(out), n, f2 // 2, *q8.args(q),
                                                  _ext.stream_ptr(gu.device)), "nd_swiglu_fwd_q")
            q8.out = q
        else:
            _ext.check(_ext.lib().nd_swiglu_fwd(_ext.ptr(gu), _ext.ptr(out), _ext.dtcode(gu), n, f2 // 2,
                                                _ext.stream_ptr(gu.device)), "nd_swiglu_fwd")
        ctx.save_for_backward(gu)
        ctx.q8_bwd = q8_bwd if gu.dtype == torch.bfloat16 else None
        return out

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        dy = dy.contiguous()
        n, f2 = gu.shape
        dgu = torch.empty_like(gu)
        if ctx.q8_bwd is not None:
            q = ctx.q8_bwd.alloc((n, f2), gu.device)
            _ext.check(_ext.lib().nd_swiglu_bwd_q(_ext.ptr(dy), _ext.ptr(gu), _ext.ptr(dgu), n, f2 // 2,
                                                  *ctx.q8_bwd.args(q), _ext.stream_ptr(gu.device)), "nd_swiglu_bwd_q")
            ctx.q8_bwd.stash(dgu, q)
        else:
            _ext.check(_ext.lib().nd_swiglu_bwd(_ext.ptr(dy), _ext.ptr(gu), _ext.ptr(dgu), _ext.dtcode(gu), n,
                                                f2 // 2, _ext.stream_ptr(gu.device)), "nd_swiglu_bwd")
        return dgu, None, None


def swiglu(gu: torch.Tensor, q8=None, q8_bwd=None) -> torch.Tensor:
    if _ext.use_hip(gu):
        return SwiGLUFn.apply(gu, q8, q8_bwd)
    return ref.swiglu(gu)
