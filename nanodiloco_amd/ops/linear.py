"""Projection GEMMs with gradient routing into the flat fp32 grad buffer.

``y = x @ W^T`` for W of shape [out, in].  Forward and dgrad are plain library GEMMs
(hipBLASLt through ``torch.mm``).  The weight gradient is accumulated straight into the fp32
``ParamStore.grad`` view: bf16 operands, fp32 accumulate, beta=1 -- one GEMM, no bf16 grad
tensor, no separate accumulate pass.  On the HIP path that GEMM is our own ``nd_wgrad`` kernel
(ops/gemm.py); otherwise hipBLASLt ``addmm(out_dtype=fp32)`` (this replaces autograd's per-parameter AccumulateGrad,
K11 in SURVEY.md §2.3).  Fused weights (q|k|v, gate|up) are single views, so one GEMM covers
all three / both projections.
"""
from __future__ import annotations

import torch

from . import _ext

_DTYPE_OUT_OK = {"checked": False, "ok": False}


def wgrad_accumulate(gw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor):
    """gw[out, in] (fp32) += dy[N, out]^T @ x[N, in]."""
    if dy.dtype == torch.float32:
        gw.addmm_(dy.t(), x)
        return
    if gw.is_cuda and _ext.get_backend() != "torch":
        from .gemm import wgrad, wgrad_supported
        if wgrad_supported(gw, dy, x):
            wgrad(gw, dy, x)
            return
    if gw.is_cuda:
        st = _DTYPE_OUT_OK
        if not st["checked"] or st["ok"]:
            try:
                torch.ops.aten.addmm.dtype_out(gw, dy.t(), x, torch.float32, beta=1, alpha=1, out=gw)
                st["checked"], st["ok"] = True, True
                return
            except (RuntimeError, NotImplementedError):
                st["checked"], st["ok"] = True, False
    gw.add_(torch.mm(dy.t(), x).float())


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, gw):
        ctx.save_for_backward(x, w)
        ctx.gw = gw
        return torch.mm(x, w.t())

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.mm(dy, w) if ctx.needs_input_grad[0] else None
        if ctx.gw is not None:
            wgrad_accumulate(ctx.gw, dy, x)
        return dx, None, None


def linear(x: torch.Tensor, w: torch.Tensor, gw: torch.Tensor) -> torch.Tensor:
    return LinearFn.apply(x, w, gw)
