"""Projection GEMMs with gradient routing into the flat fp32 grad buffer.

``y = x @ W^T`` for W of shape [out, in].  Forward and dgrad are plain library GEMMs
(hipBLASLt through ``torch.mm``).  The weight gradient is accumulated straight into the fp32
``ParamStore.grad`` view: bf16 operands, fp32 accumulate, beta=1 -- one GEMM, no bf16 grad
tensor, no separate accumulate pass.  On the HIP path that GEMM is our own ``nd_wgrad`` kernel
(ops/gemm.py); otherwise hipBLASLt ``addmm(out_dtype=fp32)`` (this replaces autograd's per-parameter AccumulateGrad,
K11 in SURVEY.md §2.3).  Fused weights (q|k|v, gate|up) are single views, so one GEMM covers
all three / both projections.

Weight-gradient overlap (``set_wgrad_overlap(True)``): the wgrad GEMM is off the backward's
critical path (nothing downstream reads it until the optimizer), so it is issued on a side HIP
stream forked from the compute stream at that point; the dgrad chain (dgrad GEMM -> SwiGLU /
RMSNorm / attention backward, several of them HBM-bound) continues on the compute stream and the
hardware co-schedules the two queues.  The compute stream joins the side stream at the end of the
backward (``join_wgrad``: embedding backward, inner-DDP layer hooks, optimizer step) -- a GPU-side
wait, never a host sync.  dY / X stay referenced until that join (then the compute stream, which
allocated them, is ordered after the side stream, so the caching allocator may reuse them at once;
``record_stream`` instead defers every such free behind an event and made the allocator fall
back to fresh hipMalloc calls -- host stalls of hundreds of ms per step).

GEMM fence: the compute stream also joins before every LIBRARY GEMM (``library_gemm_fence``).
hipBLASLt's stream-K kernels keep one workgroup per CU and make workgroups wait on each other's
partial tiles; when a side-stream wgrad holds CUs, part of that grid cannot become resident and
the resident part spins -- measured 2-8x slower steps.  Fenced, a wgrad co-runs only with our own
kernels (SwiGLU / RMSNorm backward, the attention backward), which never wait on each other.
"""
from __future__ import annotations

import torch

from . import _ext

_DTYPE_OUT_OK = {"checked": False, "ok": False}
_OVERLAP = {"enabled": False, "fence": True, "streams": {}, "pending": set(), "keep": []}
_DGRAD_T = {"enabled": True}


def transpose_into(dst: torch.Tensor, w: torch.Tensor) -> None:
    """dst[in, out] = w[out, in]^T (bf16 HIP kernel on the GPU; strided copy otherwise)."""
    if w.is_cuda and w.dtype == torch.bfloat16 and _ext.get_backend() != "torch":
        _ext.check(_ext.lib().nd_transpose_bf16(_ext.ptr(w), _ext.ptr(dst), w.shape[0], w.shape[1], w.stride(0),
                                                 dst.stride(0), _ext.stream_ptr(w.device)), "nd_transpose_bf16")
    else:
        dst.copy_(w.t())


def set_dgrad_transposed(enabled: bool) -> None:
    """Input-gradient GEMMs read a transposed weight copy (see ``LinearFn``)."""
    _DGRAD_T["enabled"] = bool(enabled)


def dgrad_transposed_enabled() -> bool:
    return _DGRAD_T["enabled"]


def set_wgrad_overlap(mode) -> None:
    """Issue projection weight-gradient GEMMs on a side stream (GPU only).  0/False: off;
    1/True: on, fenced before every library GEMM; 2: on, unfenced (A/B only, see module doc)."""
    _OVERLAP["enabled"] = int(mode) != 0
    _OVERLAP["fence"] = int(mode) != 2


def wgrad_overlap_enabled() -> bool:
    return _OVERLAP["enabled"]


def _side_stream(device: torch.device) -> torch.cuda.Stream:
    key = device.index if device.index is not None else torch.cuda.current_device()
    s = _OVERLAP["streams"].get(key)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _OVERLAP["streams"][key] = s
    return s


def join_wgrad(device=None) -> None:
    """Make the current stream wait for every weight-gradient GEMM issued on the side stream
    (no-op when nothing is outstanding)."""
    if not _OVERLAP["pending"]:
        return
    keys = list(_OVERLAP["pending"]) if device is None else [
        torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()]
    for k in keys:
        if k in _OVERLAP["pending"]:
            torch.cuda.current_stream(k).wait_stream(_OVERLAP["streams"][k])
            _OVERLAP["pending"].discard(k)
    if not _OVERLAP["pending"]:
        _OVERLAP["keep"].clear()  # operands of the joined wgrads: safe to free on the compute stream


def library_gemm_fence(device=None) -> None:
    """Call right before a hipBLASLt GEMM on the compute stream (see module doc: GEMM fence)."""
    if _OVERLAP["pending"] and _OVERLAP["fence"]:
        join_wgrad(device)


def _wgrad_on_side_stream(gw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> None:
    cur = torch.cuda.current_stream(gw.device)
    side = _side_stream(gw.device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        wgrad_accumulate(gw, dy, x)
    _OVERLAP["keep"].append((dy, x))
    _OVERLAP["pending"].add(side.device.index)


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
    """``wt`` (optional) is W^T stored [in, out] contiguous: the input gradient is then dY . (W^T)^T,
    the same K-contiguous "NT" operand layout as the forward GEMM, which hipBLASLt runs 14-16 %
    faster than dY . W (row-major x row-major) on every Llama-150M shape
    (scripts/dgrad_layout_bench.py); the model keeps the copies in step with the optimizer."""

    @staticmethod
    def forward(ctx, x, w, gw, wt=None):
        ctx.save_for_backward(x, w if wt is None else wt)
        ctx.gw = gw
        ctx.transposed = wt is not None
        library_gemm_fence(x.device if x.is_cuda else None)
        return torch.mm(x, w.t())

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        if ctx.needs_input_grad[0]:
            library_gemm_fence(dy.device if dy.is_cuda else None)
            dx = torch.mm(dy, w.t()) if ctx.transposed else torch.mm(dy, w)
        else:
            dx = None
        if ctx.gw is not None:
            if _OVERLAP["enabled"] and ctx.gw.is_cuda:
                _wgrad_on_side_stream(ctx.gw, dy, x)
            else:
                wgrad_accumulate(ctx.gw, dy, x)
        return dx, None, None, None


def linear(x: torch.Tensor, w: torch.Tensor, gw: torch.Tensor, wt: torch.Tensor = None) -> torch.Tensor:
    return LinearFn.apply(x, w, gw, wt)


_FUSED_SWIGLU = {"enabled": False}


def set_fused_swiglu(enabled: bool) -> None:
    """gate|up projection + SwiGLU as one own-GEMM launch with the activation in its epilogue
    (``LinearSwiGLUFn``) vs the tuned hipBLASLt GEMM + ``swiglu_fwd`` kernel (default).  Off by
    default: 1.05-1.08x in isolation against untuned hipBLASLt, but -0.9 % end to end against the
    pre-tuned table (bench.py --fused-swiglu 1: 731k vs 738k tok/s, 2 interleaved rounds)."""
    _FUSED_SWIGLU["enabled"] = bool(enabled)


def fused_swiglu_enabled() -> bool:
    return _FUSED_SWIGLU["enabled"]


def linear_swiglu_supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    from .gemm import nt_supported
    return (_FUSED_SWIGLU["enabled"] and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2
            and nt_supported(x, w) and (w.shape[0] // 2) % 8 == 0)


class LinearSwiGLUFn(torch.autograd.Function):
    """act = silu(x W_g^T) * (x W_u^T) for the fused [W_gate; W_up] weight: the own projection GEMM
    (csrc/gemm.hip, EPI_SWIGLU) writes gu = [gate | up] (the backward's input) and act from its
    accumulators -- no separate SwiGLU pass over gu (measured 1.05-1.08x the hipBLASLt GEMM +
    swiglu_fwd pair, profiles/r2_gemm_ab.md).  Backward: ``nd_swiglu_bwd`` -> the usual dgrad /
    wgrad of the fused projection (ops/linear.py semantics: W^T copy, side-stream wgrad)."""

    @staticmethod
    def forward(ctx, x, w, gw, wt=None):
        from .gemm import gemm_nt_swiglu
        gu, act = gemm_nt_swiglu(x, w)
        ctx.save_for_backward(x, w if wt is None else wt, gu)
        ctx.gw = gw
        ctx.transposed = wt is not None
        return act

    @staticmethod
    def backward(ctx, dact):
        x, w, gu = ctx.saved_tensors
        dact = dact.contiguous()
        n, f2 = gu.shape
        dgu = torch.empty_like(gu)
        _ext.check(_ext.lib().nd_swiglu_bwd(_ext.ptr(dact), _ext.ptr(gu), _ext.ptr(dgu), _ext.dtcode(gu), n, f2 // 2,
                                            _ext.stream_ptr(gu.device)), "nd_swiglu_bwd")
        dx = None
        if ctx.needs_input_grad[0]:
            library_gemm_fence(dgu.device)
            dx = torch.mm(dgu, w.t()) if ctx.transposed else torch.mm(dgu, w)
        if ctx.gw is not None:
            if _OVERLAP["enabled"]:
                _wgrad_on_side_stream(ctx.gw, dgu, x)
            else:
                wgrad_accumulate(ctx.gw, dgu, x)
        return dx, None, None, None


def linear_swiglu(x: torch.Tensor, w: torch.Tensor, gw: torch.Tensor, wt: torch.Tensor = None) -> torch.Tensor:
    return LinearSwiGLUFn.apply(x, w, gw, wt)
