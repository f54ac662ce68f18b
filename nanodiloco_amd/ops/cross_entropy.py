"""Fused lm_head + cross-entropy with the backward computed during the forward (K9).

The reference materialises fp32 logits ``[N, V]`` and their gradient (1.05 GB each per 8k-token
micro-batch; 33.5 GB at 262k tokens).  Here the N rows are processed in
chunks; for each chunk:

  1. ``logits = y_c @ W^T``            (the plain projection GEMM, ops.linear.mm_nt: the selected
                                       --proj-gemm kernel; compute dtype)
  2. ``nd_ce_fwd_bwd``                 one HIP kernel, one row per workgroup: online max/sum-exp over V,
                                       per-row loss summed into a device scalar, and the logits
                                       buffer overwritten IN PLACE by ``dlogits = (softmax - onehot) * s``
  3. ``dy_c = dlogits @ W``            (dgrad, kept for backward)
  4. ``gW += dlogits^T @ y_c``         (wgrad, fp32 accumulate into the flat grad buffer)

so only one chunk of logits ever exists and nothing [N, V]-sized survives the forward.
``s = loss_scale / n_valid`` is read from device memory (no host sync).

fp8 (``f8`` = the model's ``Fp8Linears``, BASELINE config 5): the three GEMMs run on the own fp8 kernels --
logits = e4m3 y8 . W8^T, the CE kernel writes the dlogits straight as e5m2 (delayed scaling, slot "x.lm";
``nd_ce_fwd_bwd_q8``, bitwise the bf16 dlogits + separate cast that the first step, which has no scale yet,
still takes), dy = dlogits8 . (W^T)8^T and gW += dlogits8^T y8 (wgrad8_pp_kernel).  The returned loss is the
unscaled mean over valid tokens (ignore_index=-100), matching ``HF/loss/loss_utils.py:32-71``.

Contract: the weight gradient is produced in the forward, assuming the loss is back-propagated
with unit upstream gradient (``loss.backward()``); ``loss_scale`` is how callers scale it
(e.g. 1/grad_accum).  The activation gradient is additionally multiplied by the upstream
gradient, so ``dy`` is correct for any upstream value.
"""
from __future__ import annotations

import os

import torch

from . import _ext
from .determinism import deterministic
from .linear import mm_nt, wgrad_accumulate

IGNORE_INDEX = -100
_HIP_INVALID_VALUE = 1  # hipErrorInvalidValue: a launcher refused the shape (caller takes the general path)


# logits chunk budget (ND_CE_CHUNK_MB, default 4 GiB: a whole 64k-token micro-batch of a 32k
# vocabulary in bf16 -- one GEMM triple per micro-batch; +0.35 % over 1 GiB chunks, profiles/r2_ce_chunk_ab.md)
_CHUNK_BYTES = int(float(os.environ.get("ND_CE_CHUNK_MB", "4096")) * (1 << 20))


def _chunk_rows(V: int, elem: int, budget_bytes: int = 0) -> int:
    return max(256, ((budget_bytes or _CHUNK_BYTES) // (V * elem)) // 256 * 256)


class LMHeadCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, w, gw, targets, loss_scale, chunk_rows, wt, f8=None):
        n, d = y.shape
        V = w.shape[0]
        targets = targets.reshape(-1)
        valid = (targets != IGNORE_INDEX).sum().to(torch.float32)
        denom = valid.clamp_min(1.0)
        scale = (loss_scale / denom).reshape(1).contiguous()
        dy = torch.empty_like(y)
        loss_sum = torch.zeros(1, dtype=torch.float32, device=y.device)
        hip = _ext.use_hip(y)
        det = deterministic()
        q = None
        if f8 is not None and hip:
            from .fp8 import E4M3, E5M2, _wgrad_f8, cast
            from .gemm import gemm_pp_f8, pp_f8_supported
            lin, version, y8 = f8
            kx, kdy = lin._slots(LM_KEY)
            r = lin.recipe
            if y8 is None or y8.shape != y.shape:
                y8 = r.quantize(y, kx, E4M3)
            wq = lin.weights[LM_KEY].get(w, version)
            if pp_f8_supported(y8, wq.w8) and V % 128 == 0:
                q = (r, kx, kdy, y8, wq)
        chunk = chunk_rows or _chunk_rows(V, y.element_size() if hip else 4)
        if not chunk_rows and n > chunk:  # equal-sized chunks: one GEMM shape, one tuned kernel
            nch = -(-n // chunk)
            chunk = (-(-n // nch) + 255) // 256 * 256
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            yc, tc = y[s:e], targets[s:e]
            if hip:
                if q is not None:  # fp8: e4m3 x e4m3 on the own fp8 ping-pong kernel
                    r, kx, kdy, y8, wq = q
                    logits = gemm_pp_f8(y8[s:e], wq.w8, r.inv[kx:kx + 1], wq.inv)
                else:  # the selected plain projection GEMM (ops/linear.py proj_gemm: hipBLASLt by default)
                    logits = mm_nt(yc, w)
                rows = torch.empty(e - s, dtype=torch.float32, device=y.device) if det else None
                dl8 = None
                t8 = q[0].target(q[2], E5M2) if q is not None else None
                if t8 is not None:
                    # fp8: the CE kernel writes the e5m2 dlogits itself (no bf16 dlogits, no separate cast)
                    q8 = t8.alloc((e - s, V), y.device)
                    rc = _ext.lib().nd_ce_fwd_bwd_q8(_ext.ptr(logits), _ext.dtcode(logits), _ext.ptr(tc),
                                                     _ext.ptr(loss_sum), _ext.ptr(scale), e - s, V, IGNORE_INDEX, 0,
                                                     _ext.ptr(rows) if det else 0, *t8.args(q8),
                                                     _ext.stream_ptr(y.device))
                    if rc == 0:
                        dl8 = q8
                    elif rc != _HIP_INVALID_VALUE:  # invalid value = shape not taken: cast separately below
                        _ext.check(rc, "nd_ce_fwd_bwd_q8")
                if dl8 is None:
                    _ext.check(_ext.lib().nd_ce_fwd_bwd(_ext.ptr(logits), _ext.dtcode(logits), _ext.ptr(tc),
                                                        _ext.ptr(loss_sum), _ext.ptr(scale), e - s, V, IGNORE_INDEX,
                                                        0, _ext.ptr(rows) if det else 0, 0.0,
                                                        _ext.stream_ptr(y.device)), "nd_ce_fwd_bwd")
                if det:  # per-row losses, one ordered reduction (no float atomics)
                    loss_sum += rows.sum()
                dl = logits if dl8 is None else None
            else:
                dl8 = None
                logits = torch.mm(yc.float(), w.float().t())
                lse = torch.logsumexp(logits, dim=-1)
                ok = tc != IGNORE_INDEX
                tgt = torch.where(ok, tc, torch.zeros_like(tc))
                picked = logits.gather(1, tgt[:, None])[:, 0]
                loss_sum += torch.where(ok, lse - picked, torch.zeros_like(lse)).sum()
                p = torch.softmax(logits, dim=-1)
                p.scatter_add_(1, tgt[:, None], -torch.ones_like(p[:, :1]))
                p *= ok[:, None].to(p.dtype) * scale
                dl = p.to(y.dtype)
            if q is not None:
                # e5m2 dlogits (one cast; delayed scaling of slot kdy), then both gradient GEMMs in fp8
                r, kx, kdy, y8, wq = q
                if dl8 is None:
                    r._first_use(dl, kdy)
                    dl8 = cast(dl, r.scale[kdy:kdy + 1], E5M2, r.amax[kdy])
                gemm_pp_f8(dl8, wq.wT8, r.inv[kdy:kdy + 1], wq.inv, out=dy[s:e])
                if gw is not None:
                    _wgrad_f8(gw, dl8, y8[s:e], r.inv[kdy:kdy + 1], r.inv[kx:kx + 1], dl)
                continue
            # dy rows written in place (a row slice of a contiguous tensor); with wt = W^T the GEMM
            # has the faster K-contiguous operand layout (ops/linear.py)
            if wt is not None and dl.dtype == wt.dtype:
                mm_nt(dl, wt, out=dy[s:e])
            elif dl.dtype == w.dtype:
                torch.mm(dl, w, out=dy[s:e])
            else:
                dy[s:e] = torch.mm(dl, w.to(dl.dtype))
            if gw is not None:
                # stays on the compute stream: the chunk loop is GEMM-bound (library GEMMs fence
                # side-stream work anyway, ops/linear.py)
                wgrad_accumulate(gw, dl, yc.to(dl.dtype))
        ctx.save_for_backward(dy)
        return (loss_sum / denom).reshape(())

    @staticmethod
    def backward(ctx, g):
        (dy,) = ctx.saved_tensors
        return dy * g.to(dy.dtype), None, None, None, None, None, None, None


LM_KEY = "x.lm"  # the lm head's slot pair / weight cache in Fp8Linears (ops/fp8.py fp8_projection("lm"))


def lm_head_ce(y: torch.Tensor, w: torch.Tensor, gw: torch.Tensor, targets: torch.Tensor,
               loss_scale: float = 1.0, chunk_rows: int = 0, wt: torch.Tensor = None, f8=None) -> torch.Tensor:
    """``wt``: optional W^T copy [d, V] for the input-gradient GEMM (see ops/linear.py).  ``f8``:
    (Fp8Linears, weight version, fused e4m3 copy of y or None) for the fp8 lm head."""
    return LMHeadCEFn.apply(y, w, gw, targets, float(loss_scale), int(chunk_rows), wt, f8)
