"""Weight-gradient GEMM on the HIP path (``nd_wgrad``): ``gW[M, N] (fp32) += dY[K, M]^T @ X[K, N]``.

hipBLASLt runs this token-reduction layout at 330-900 TF/s on the Llama-150M shapes (profiles/),
because K (tokens) is the strided axis of both operands; the custom kernel stages both operands
through LDS as they lie in memory and forms MFMA fragments with transposing LDS reads, with a
deterministic split-K for the small outputs.  Plain fwd / dgrad GEMMs stay on hipBLASLt.
"""
from __future__ import annotations

import torch

from . import _ext

_WS = {}


def _workspace(device, numel):
    """Split-K slab workspace, one per (device, stream): wgrads issued on the side stream
    (ops/linear.py overlap) and on the compute stream (lm head) must not share slabs."""
    stream = torch.cuda.current_stream(device)
    key = (str(device), stream.cuda_stream)
    t = _WS.get(key)
    if t is None or t.numel() < numel:
        t = torch.empty(max(numel, 1 << 20), dtype=torch.float32, device=device)
        _WS[key] = t
    return t


def wgrad_supported(gw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> bool:
    return (gw.is_cuda and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and gw.dtype == torch.float32
            and dy.dim() == 2 and x.dim() == 2 and dy.stride(1) == 1 and x.stride(1) == 1 and gw.stride(1) == 1
            and dy.shape[1] % 8 == 0 and x.shape[1] % 8 == 0 and dy.stride(0) % 8 == 0 and x.stride(0) % 8 == 0
            and gw.stride(0) % 4 == 0)


def wgrad(gw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> None:
    K, M = dy.shape
    N = x.shape[1]
    assert x.shape[0] == K and tuple(gw.shape) == (M, N)
    L = _ext.lib()
    S = L.nd_wgrad_splits(M, N, K)
    ws = _workspace(gw.device, S * M * N) if S > 1 else None
    _ext.check(L.nd_wgrad(_ext.ptr(dy), _ext.ptr(x), _ext.ptr(gw), _ext.ptr(ws), M, N, K, dy.stride(0), x.stride(0),
                          gw.stride(0), _ext.stream_ptr(gw.device)), "nd_wgrad")
