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
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        n, f2 = gu.shape
        out = torch.empty(n, f2 // 2, dtype=gu.dtype, device=gu.device)
        _ext.check(_ext.lib().nd_swiglu_fwd(_ext.ptr(gu), _ext.ptr(out), _ext.dtcode(gu), n, f2 // 2,
                                            _ext.stream_ptr(gu.device)), "nd_swiglu_fwd")
        ctx.save_for_backward(gu)
        return out

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        dy = dy.contiguous()
        n, f2 = gu.shape
        dgu = torch.empty_like(gu)
        _ext.check(_ext.lib().nd_swiglu_bwd(_ext.ptr(dy), _ext.ptr(gu), _ext.ptr(dgu), _ext.dtcode(gu), n, f2 // 2,
                                            _ext.stream_ptr(gu.device)), "nd_swiglu_bwd")
        return dgu


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    if _ext.use_hip(gu):
        return SwiGLUFn.apply(gu)
    return ref.swiglu(gu)
