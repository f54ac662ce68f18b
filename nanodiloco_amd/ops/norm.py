"""RMSNorm and residual-add + RMSNorm with gradient routing.

Residual stream is kept in fp32 by default (what HF bf16-autocast effectively does: the embedding output is
fp32 and every residual add promotes), norm weights are read from the fp32 master, the
normalised output is emitted in the compute dtype for the next GEMM.  A bf16 residual stream
(``--residual-dtype bf16``) is the same ops on a bf16 ``h``: h_new is rounded to bf16 before the
statistics, the residual gradient is bf16 and doubles as the branch gradient (docs/DESIGN.md, norm passes).

Forward, HIP path: one kernel, one row per wave (``nd_rmsnorm_fwd``) fusing
``h_new = h + a`` (K8) with ``y = w * h_new * rstd`` (K2) and saving ``rstd``.
Backward: one kernel producing dx (in the residual dtype, already summed with the incoming residual
grad) and the branch grad in the compute dtype (the same tensor as dx for a bf16 residual), plus
per-block dw partials that are reduced into the flat grad buffer.
"""
from __future__ import annotations

import torch

from . import _ext
from . import reference as ref


def _rows(x):
    return x.reshape(-1, x.shape[-1])


def _q8_ok(q8, x, a, out_dtype):
    return (q8 is not None and out_dtype == torch.bfloat16 and x.dtype in (torch.float32, torch.bfloat16)
            and (a is None or a.dtype == torch.bfloat16))


def _hip_fwd(x, a, w, eps, out_dtype, q8=None):
    """``q8`` (ops/fp8.QuantTarget): also write the fp8 copy of y (set as ``q8.out``)."""
    x2 = _rows(x)
    rows, cols = x2.shape
    y = torch.empty(rows, cols, dtype=out_dtype, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    h = torch.empty(rows, cols, dtype=x.dtype, device=x.device) if a is not None else None
    L = _ext.lib()
    common = (_ext.ptr(x2), _ext.dtcode(x2), _ext.ptr(a), _ext.dtcode(a) if a is not None else 0,
              _ext.ptr(w), _ext.ptr(y), _ext.dtcode(y), _ext.ptr(h), _ext.ptr(rstd), rows, cols, float(eps))
    if _q8_ok(q8, x2, a, out_dtype):
        q = q8.alloc((rows, cols), x.device)
        _ext.check(L.nd_rmsnorm_fwd_q(*common, *q8.args(q), _ext.stream_ptr(x.device)), "nd_rmsnorm_fwd_q")
        q8.out = q
    else:
        _ext.check(L.nd_rmsnorm_fwd(*common, _ext.stream_ptr(x.device)), "nd_rmsnorm_fwd")
    return y, (h if h is not None else x2), rstd


def _hip_bwd(dy, hx, w, rstd, dres, gw, branch_dtype, q8_bwd=None):
    """``q8_bwd`` (ops/fp8.QuantTarget): also write the fp8 copy of the branch gradient (stashed for
    the projection whose output it is the gradient of)."""
    rows, cols = hx.shape
    dx = torch.empty(rows, cols, dtype=hx.dtype, device=hx.device)
    if branch_dtype is not None and hx.dtype == torch.bfloat16 and branch_dtype == torch.bfloat16:
        da = dx  # bf16 residual: the residual gradient IS the branch gradient (one store)
    else:
        da = torch.empty(rows, cols, dtype=branch_dtype, device=hx.device) if branch_dtype is not None else None
    nblk = min(1024, (rows + 63) // 64)
    part = torch.empty(nblk, cols, dtype=torch.float32, device=hx.device)
    L = _ext.lib()
    dy2 = _rows(dy).contiguous()
    if dres is not None and dres.dtype != hx.dtype:
        dres = dres.to(hx.dtype)
    common = (_ext.ptr(dy2), _ext.dtcode(dy2), _ext.ptr(hx), _ext.dtcode(hx), _ext.ptr(w), _ext.ptr(rstd),
              _ext.ptr(dres), _ext.ptr(dx), _ext.dtcode(da) if da is not None else 0,
              _ext.ptr(da), rows, cols, _ext.ptr(part))
    if q8_bwd is not None and da is not None and da.dtype == torch.bfloat16 and dy2.dtype == torch.bfloat16:
        q = q8_bwd.alloc((rows, cols), hx.device)
        _ext.check(L.nd_rmsnorm_bwd_q(*common, *q8_bwd.args(q), _ext.stream_ptr(hx.device)), "nd_rmsnorm_bwd_q")
        q8_bwd.stash(da, q)
    else:
        _ext.check(L.nd_rmsnorm_bwd(*common, _ext.stream_ptr(hx.device)), "nd_rmsnorm_bwd")
    if gw is not None:
        _ext.check(L.nd_colsum_add(_ext.ptr(part), _ext.ptr(gw), nblk, cols, _ext.stream_ptr(hx.device)),
                   "nd_colsum_add")
    return dx, da


class RMSNormFn(torch.autograd.Function):
    """y = rmsnorm(x) * w ; x is the (fp32) residual stream."""

    @staticmethod
    def forward(ctx, x, w, gw, eps, out_dtype, q8=None):
        ctx.eps, ctx.gw, ctx.shape = eps, gw, x.shape
        if _ext.use_hip(x):
            y, hx, rstd = _hip_fwd(x, None, w, eps, out_dtype, q8)
            ctx.save_for_backward(hx, w, rstd)
            ctx.hip = True
            return y.view(*x.shape[:-1], x.shape[-1])
        ctx.hip = False
        ctx.save_for_backward(x, w)
        return ref.rmsnorm(x.float(), w, eps).to(out_dtype)

    @staticmethod
    def backward(ctx, dy):
        if ctx.hip:
            hx, w, rstd = ctx.saved_tensors
            dx, _ = _hip_bwd(dy, hx, w, rstd, None, ctx.gw, None)
            return dx.view(ctx.shape), None, None, None, None, None
        x, w = ctx.saved_tensors
        dx, dw = ref.rmsnorm_backward(dy, x, w, ctx.eps)
        if ctx.gw is not None:
            ctx.gw.add_(dw)
        return dx.to(x.dtype), None, None, None, None, None


class RMSNormResFn(torch.autograd.Function):
    """y = rmsnorm(x) * w, also returning x itself (as a view) for the residual stream.  Used for the
    first norm, whose input (the embedding output) also starts the residual path: routing both uses
    through this one node lets the backward kernel add the residual gradient (``dres``) in place of a
    separate autograd accumulation, a full fp32 [N, d] read-read-write pass per micro-batch."""

    @staticmethod
    def forward(ctx, x, w, gw, eps, out_dtype, q8=None):
        ctx.set_materialize_grads(False)
        ctx.eps, ctx.gw, ctx.shape, ctx.y_dtype = eps, gw, x.shape, out_dtype
        if _ext.use_hip(x):
            y, hx, rstd = _hip_fwd(x.contiguous(), None, w, eps, out_dtype, q8)
            ctx.save_for_backward(hx, w, rstd)
            ctx.hip = True
            return y.view(x.shape), x.view_as(x)
        ctx.hip = False
        ctx.save_for_backward(x, w)
        return ref.rmsnorm(x.float(), w, eps).to(out_dtype), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dres):
        if dy is None:
            dy = torch.zeros(ctx.shape, dtype=ctx.y_dtype, device=ctx.saved_tensors[0].device)
        if ctx.hip:
            hx, w, rstd = ctx.saved_tensors
            dr = _rows(dres).to(hx.dtype).contiguous() if dres is not None else None
            dx, _ = _hip_bwd(dy, hx, w, rstd, dr, ctx.gw, None)
            return dx.view(ctx.shape), None, None, None, None, None
        x, w = ctx.saved_tensors
        dx, dw = ref.rmsnorm_backward(dy, x, w, ctx.eps)
        if dres is not None:
            dx = dx + dres.float()
        if ctx.gw is not None:
            ctx.gw.add_(dw)
        return dx.to(x.dtype), None, None, None, None, None


class AddRMSNormFn(torch.autograd.Function):
    """h_new = h + a ; y = rmsnorm(h_new) * w.  Returns (y, h_new)."""

    @staticmethod
    def forward(ctx, h, a, w, gw, eps, out_dtype, q8=None, q8_bwd=None):
        # the final norm's h_new output is unused: keep its gradient None instead of a zero-filled
        # [N, d] fp32 tensor (a fill plus a full extra read in the backward kernel)
        ctx.set_materialize_grads(False)
        ctx.eps, ctx.gw, ctx.shape, ctx.a_dtype, ctx.y_dtype, ctx.h_dtype = eps, gw, h.shape, a.dtype, out_dtype, h.dtype
        if _ext.use_hip(h):
            y, hn, rstd = _hip_fwd(h, _rows(a).contiguous(), w, eps, out_dtype, q8)
            ctx.save_for_backward(hn, w, rstd)
            ctx.hip = True
            ctx.q8_bwd = q8_bwd
            return y.view(h.shape), hn.view(h.shape)
        ctx.hip = False
        hn = h.float() + a.float()
        if h.dtype != torch.float32:  # bf16 residual: statistics of the stored (rounded) h_new
            hn = hn.to(h.dtype).float()
        ctx.save_for_backward(hn, w)
        return ref.rmsnorm(hn, w, eps).to(out_dtype), hn.to(h.dtype)

    @staticmethod
    def backward(ctx, dy, dhn):
        if dy is None:
            dy = torch.zeros(ctx.shape, dtype=ctx.y_dtype, device=ctx.saved_tensors[0].device)
        if ctx.hip:
            hn, w, rstd = ctx.saved_tensors
            dres = _rows(dhn).contiguous() if dhn is not None else None
            dx, da = _hip_bwd(dy, hn, w, rstd, dres, ctx.gw, ctx.a_dtype, ctx.q8_bwd)
            # bf16 residual: dx and da are ONE tensor; both consumers (the previous norm's dres, the projection's
            # dgrad / wgrad) only read it, and neither input is used twice, so autograd never accumulates into it
            return dx.view(ctx.shape), da.view(ctx.shape), None, None, None, None, None, None
        hn, w = ctx.saved_tensors
        dx, dw = ref.rmsnorm_backward(dy, hn, w, ctx.eps)
        if dhn is not None:
            dx = dx + dhn.float()
        if ctx.gw is not None:
            ctx.gw.add_(dw)
        if ctx.h_dtype != torch.float32:
            dx = dx.to(ctx.h_dtype)
        return dx, dx.to(ctx.a_dtype), None, None, None, None, None, None


def rmsnorm(x, w, gw, eps, out_dtype=None, q8=None):
    """``q8`` (fp8 inner step): fused fp8 copy of the output for the next projection (ops/fp8.py)."""
    return RMSNormFn.apply(x, w, gw, eps, out_dtype or x.dtype, q8)


def rmsnorm_res(x, w, gw, eps, out_dtype=None, q8=None):
    """(y, x): ``rmsnorm`` plus a pass-through of ``x`` whose gradient is fused into this op's
    backward kernel; use when ``x`` also feeds the residual stream."""
    return RMSNormResFn.apply(x, w, gw, eps, out_dtype or x.dtype, q8)


def add_rmsnorm(h, a, w, gw, eps, out_dtype=None, q8=None, q8_bwd=None):
    """``q8`` / ``q8_bwd`` (fp8 inner step): fused fp8 copies of y (next projection's input) and of
    the branch gradient (the gradient of the projection that produced ``a``); see ops/fp8.py."""
    return AddRMSNormFn.apply(h, a, w, gw, eps, out_dtype or a.dtype, q8, q8_bwd)
