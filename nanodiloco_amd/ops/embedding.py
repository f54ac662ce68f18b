"""Token embedding (K1): gather rows of the fp32 master table into the residual stream (fp32, or bf16 for
``--residual-dtype bf16``: rounded in the gather, no separate cast pass); backward scatter-adds the residual
gradient rows (fp32 or bf16) into the flat fp32 grad buffer.

HIP path: ``nd_embedding_fwd`` (one wave per token row, 16-B vector loads) and
``nd_embedding_bwd`` (one wave per token row, f32 atomics on whole contiguous rows -- the
access shape the MI355X atomic unit serves at full rate, MI355X_MICROARCH.md §Global float atomics),
or, in deterministic mode (ops/determinism.py), ``nd_embedding_bwd_sorted`` over a stable argsort
(fixed 64-row chunks of the sorted order plus an ordered join of the runs that cross chunks, so a
long run of one pad id does not serialise on one wave).
"""
from __future__ import annotations

import torch

from . import _ext
from .determinism import deterministic


class EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w, gw, anchor, out_dtype=None):
        ids = ids.reshape(-1)
        ctx.save_for_backward(ids)
        ctx.gw = gw
        ctx.vocab = w.shape[0]
        odt = out_dtype or w.dtype
        if _ext.use_hip(w) and w.dtype == torch.float32:
            n, d = ids.numel(), w.shape[1]
            out = torch.empty(n, d, dtype=odt, device=w.device)
            _ext.check(_ext.lib().nd_embedding_fwd(_ext.ptr(ids), _ext.ptr(w), _ext.ptr(out), _ext.dtcode(out), n, d,
                                                   w.shape[0], _ext.stream_ptr(w.device)), "nd_embedding_fwd")
            ctx.hip = True
            return out
        ctx.hip = False
        return w.index_select(0, ids).to(odt)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        if ctx.gw is not None:
            dy = dy.contiguous()
            if ctx.hip:
                n, d = dy.shape
                if deterministic():
                    perm = torch.argsort(ids, stable=True)
                    sid = ids.index_select(0, perm).contiguous()
                    ws = sorted_bwd_workspace(n, d, dy.device)
                    _ext.check(_ext.lib().nd_embedding_bwd_sorted(
                        _ext.ptr(sid), _ext.ptr(perm), _ext.ptr(dy), _ext.dtcode(dy), _ext.ptr(ctx.gw), _ext.ptr(ws),
                        n, d, ctx.vocab, _ext.stream_ptr(dy.device)), "nd_embedding_bwd_sorted")
                else:
                    _ext.check(_ext.lib().nd_embedding_bwd(_ext.ptr(ids), _ext.ptr(dy), _ext.dtcode(dy),
                                                           _ext.ptr(ctx.gw), n, d, ctx.vocab,
                                                           _ext.stream_ptr(dy.device)), "nd_embedding_bwd")
            else:
                ctx.gw.index_add_(0, ids, dy.float())
        # the embedding backward is the last op of the model's backward: join the side-stream
        # weight-gradient GEMMs here so the grad buffer is complete on the compute stream
        from .linear import join_wgrad
        join_wgrad(dy.device if dy.is_cuda else None)
        return None, None, None, None, None


_ANCHORS = {}

SORTED_CHUNK = 64  # rows of the sorted order per wave in nd_embedding_bwd_sorted (kEmbChunk)


def sorted_bwd_workspace(n, d, device):
    """Head / tail partial sums of nd_embedding_bwd_sorted: 2 * ceil(n / 64) rows of d floats."""
    return torch.empty(2 * ((n + SORTED_CHUNK - 1) // SORTED_CHUNK) * d, dtype=torch.float32, device=device)


def _anchor(device):
    """A 0-element leaf requiring grad: makes the gathered rows part of the autograd graph even
    though the table itself is not an autograd leaf (its grad is routed by hand)."""
    a = _ANCHORS.get(device)
    if a is None:
        a = torch.zeros(0, device=device, requires_grad=True)
        _ANCHORS[device] = a
    return a


def embedding(ids, w, gw, out_dtype=None):
    """``out_dtype``: dtype of the gathered rows (default: the table's)."""
    return EmbeddingFn.apply(ids, w, gw, _anchor(w.device), out_dtype)
