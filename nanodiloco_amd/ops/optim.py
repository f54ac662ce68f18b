"""Flat-buffer optimizer kernels: clip + AdamW (inner, K12-K14) and the DiLoCo outer step (K15-K17).

Inner step (reference: ``clip_grad_norm_(1.0)`` then ``AdamW.step()``,
REF/nanodiloco/diloco/diloco.py:56-60):
  ``nd_sumsq_partial``  per-block sum of squares of the flat fp32 grad
  ``nd_adamw_step``     every block re-reduces the (<=1024) partials -> global norm -> clip
                        coefficient, then one fused pass: decoupled weight decay, m/v update,
                        bias-corrected step, fp32 master write AND bf16 shadow write-out.
  Two launches total, no host sync (lr / bias corrections are kernel arguments).

Outer step (reference: per-tensor pseudo-grad + all_reduce(AVG) + SGD-Nesterov + CPU snapshot,
REF/nanodiloco/diloco/diloco.py:34-54):
  ``nd_pseudograd``     delta = theta_sync - theta_local   (fp32 or bf16 wire dtype)
  -- all-reduce(SUM) of delta, bucketed, on the comm stream --
  ``nd_outer_nesterov`` one pass per bucket: buf = m*buf + delta/W (buf = delta/W on the first
                        outer step), theta = theta_sync - lr*(delta/W + m*buf), theta_sync = theta,
                        shadow = bf16(theta); optional streaming "drift" term for the overlapped
                        mode (see parallel/diloco.py).

Every function has a PyTorch implementation with identical math (CPU path + test oracle).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from . import _ext

SUMSQ_BLOCKS = 1024


def global_grad_norm(grad: torch.Tensor) -> torch.Tensor:
    if _ext.use_hip(grad):
        part = torch.empty(SUMSQ_BLOCKS, dtype=torch.float32, device=grad.device)
        _ext.check(_ext.lib().nd_sumsq_partial(_ext.ptr(grad), grad.numel(), _ext.ptr(part), SUMSQ_BLOCKS,
                                               _ext.stream_ptr(grad.device)), "nd_sumsq_partial")
        return part.sum().sqrt()
    return grad.float().norm()


def adamw_step(master: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
               shadow: Optional[torch.Tensor], step: int, lr: float, betas=(0.9, 0.999), eps: float = 1e-8,
               weight_decay: float = 0.01, max_norm: Optional[float] = 1.0,
               norm_out: Optional[torch.Tensor] = None, skip_nonfinite: bool = False,
               skipped: Optional[torch.Tensor] = None) -> None:
    """Clip-by-global-norm + AdamW (torch.optim.AdamW semantics) over flat fp32 buffers.

    ``step`` is the 1-based AdamW step count (bias correction).  If ``norm_out`` is given, the
    pre-clip global grad norm is written to it (device scalar, for logging without a sync).
    ``skip_nonfinite``: if the global grad norm is NaN/Inf the update is skipped on the device (no
    host sync) and ``skipped`` (int32 device scalar) is incremented.
    """
    b1, b2 = betas
    bc1 = 1.0 - b1 ** step
    bc2 = 1.0 - b2 ** step
    if _ext.use_hip(master):
        n = master.numel()
        part = torch.empty(SUMSQ_BLOCKS, dtype=torch.float32, device=master.device)
        L = _ext.lib()
        s = _ext.stream_ptr(master.device)
        need_norm = max_norm is not None or norm_out is not None or skip_nonfinite
        if need_norm:
            _ext.check(L.nd_sumsq_partial(_ext.ptr(grad), n, _ext.ptr(part), SUMSQ_BLOCKS, s), "nd_sumsq_partial")
        sh = shadow if (shadow is not None and shadow.data_ptr() != master.data_ptr()) else None
        _ext.check(L.nd_adamw_step(_ext.ptr(master), _ext.ptr(grad), _ext.ptr(exp_avg), _ext.ptr(exp_avg_sq),
                                   _ext.ptr(sh), _ext.dtcode(sh) if sh is not None else 0, n,
                                   _ext.ptr(part) if need_norm else 0,
                                   SUMSQ_BLOCKS, float(lr), float(b1), float(b2), float(eps), float(weight_decay),
                                   float(bc1), float(bc2), float(max_norm if max_norm is not None else -1.0),
                                   _ext.ptr(norm_out), 1 if skip_nonfinite else 0, _ext.ptr(skipped), s),
                   "nd_adamw_step")
        return
    # ---- torch reference (same op order as torch.optim.AdamW single-tensor path)
    g = grad
    if max_norm is not None or norm_out is not None or skip_nonfinite:
        total = grad.norm()
        if norm_out is not None:
            norm_out.copy_(total.reshape(norm_out.shape))
        if skip_nonfinite and not bool(torch.isfinite(total)):
            if skipped is not None:
                skipped += 1
            return
        if max_norm is not None:
            coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
            g = grad * coef
    master.mul_(1.0 - lr * weight_decay)
    exp_avg.lerp_(g, 1.0 - b1)
    exp_avg_sq.mul_(b2).addcmul_(g, g, value=1.0 - b2)
    step_size = lr / bc1
    denom = (exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
    master.addcdiv_(exp_avg, denom, value=-step_size)
    if shadow is not None and shadow.data_ptr() != master.data_ptr():
        shadow.copy_(master)


def pseudograd(sync: torch.Tensor, master: torch.Tensor, out: torch.Tensor) -> None:
    """out = sync - master (out may be fp32 or bf16)."""
    if _ext.use_hip(master):
        _ext.check(_ext.lib().nd_pseudograd(_ext.ptr(sync), _ext.ptr(master), _ext.ptr(out), _ext.dtcode(out),
                                            master.numel(), _ext.stream_ptr(master.device)), "nd_pseudograd")
        return
    torch.sub(sync, master, out=out) if out.dtype == torch.float32 else out.copy_(sync - master)


def outer_nesterov(master: torch.Tensor, sync: torch.Tensor, delta_sum: torch.Tensor, mom: torch.Tensor,
                   shadow: Optional[torch.Tensor], inv_world: float, lr: float, momentum: float, first: bool,
                   drift_base: Optional[torch.Tensor] = None) -> None:
    """Outer SGD-Nesterov step on one (bucket) range; see module docstring.

    ``drift_base`` (fp32, optional): the pre-reduce local pseudo-gradient.  When given, the local
    progress made since the outer boundary (``master - (sync - drift_base)``) is re-applied on top
    of the new outer weights (overlapped / one-step-delayed mode).
    """
    if _ext.use_hip(master):
        sh = shadow if (shadow is not None and shadow.data_ptr() != master.data_ptr()) else None
        _ext.check(_ext.lib().nd_outer_nesterov(
            _ext.ptr(master), _ext.ptr(sync), _ext.ptr(delta_sum), _ext.dtcode(delta_sum), _ext.ptr(mom),
            _ext.ptr(sh), _ext.dtcode(sh) if sh is not None else 0, master.numel(), float(inv_world), float(lr),
            float(momentum), 1 if first else 0, _ext.ptr(drift_base), 0, _ext.stream_ptr(master.device)),
            "nd_outer_nesterov")
        return
    d = delta_sum.float() * inv_world
    if first:
        mom.copy_(d)
    else:
        mom.mul_(momentum).add_(d)
    upd = d.add(mom, alpha=momentum)
    new = sync - lr * upd
    if drift_base is not None:
        master.add_(drift_base).sub_(sync).add_(new)  # new + (local - (sync_old - drift_base))
    else:
        master.copy_(new)
    sync.copy_(new)
    if shadow is not None and shadow.data_ptr() != master.data_ptr():
        shadow.copy_(master)
