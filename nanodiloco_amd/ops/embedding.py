"""Token embedding (K1): gather rows of the fp32 master table into the fp32 residual stream;
backward scatter-adds the residual gradient rows into the flat fp32 grad buffer.

HIP path: ``nd_embedding_fwd`` (one wave per token row, 16-B vector loads) and
``nd_embedding_bwd`` (one wave per token row, f32 atomics on whole contiguous rows -- the
access shape the MI355X atomic unit serves at full rate, MI355X_MICROARCH.md §Global float atomics),
or, in deterministic mode (ops/determinism.py), ``nd_embedding_bwd_sorted`` over a stable argsort.
"""
from __future__ import annotations

import torch

from . import _ext
from .determinism import deterministic


class EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w, gw, anchor):
        ids = ids.reshape(-1)
        ctx.save_for_backward(ids)
        ctx.gw = gw
        ctx.vocab = w.shape[0]
        if _ext.use_hip(w):
            n, d = ids.numel(), w.shape[1]
            out = torch.empty(n, d, dtype=w.dtype, device=w.device)
            _ext.check(_ext.lib().nd_embedding_fwd(_ext.ptr(ids), _ext.ptr(w), _ext.ptr(out), n, d, w.shape[0],
                                                   _ext.stream_ptr(w.device)), "nd_embedding_fwd")
            ctx.hip = True
            return out
        ctx.hip = False
        return w.index_select(0, ids)

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
                    _ext.check(_ext.lib().nd_embedding_bwd_sorted(_ext.ptr(sid), _ext.ptr(perm), _ext.ptr(dy),
                                                                  _ext.ptr(ctx.gw), n, d, ctx.vocab,
                                                                  _ext.stream_ptr(dy.device)), "nd_embedding_bwd_sorted")
                else:
                    _ext.check(_ext.lib().nd_embedding_bwd(_ext.ptr(ids), _ext.ptr(dy), _ext.ptr(ctx.gw), n, d,
                                                           ctx.vocab, _ext.stream_ptr(dy.device)), "nd_embedding_bwd")
            else:
                ctx.gw.index_add_(0, ids, dy.float())
        # the embedding backward is the last op of the model's backward: join the side-stream
        # weight-gradient GEMMs here so the grad buffer is complete on the compute stream
        from .linear import join_wgrad
        join_wgrad(dy.device if dy.is_cuda else None)
        return None, None, None, None


_ANCHORS = {}


def _anchor(device):
    """A 0-element leaf requiring grad: makes the gathered rows part of the autograd graph even
    though the table itself is not an autograd leaf (its grad is routed by hand)."""
    a = _ANCHORS.get(device)
    if a is None:
        a = torch.zeros(0, device=device, requires_grad=True)
        _ANCHORS[device] = a
    return a


def embedding(ids, w, gw):
    return EmbeddingFn.apply(ids, w, gw, _anchor(w.device))
