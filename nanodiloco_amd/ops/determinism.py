"""Bitwise-reproducible mode.

Every kernel of the default step is already order-fixed (split-K weight gradients through slabs
summed in a fixed order, attention backward without atomics, column-sum RMSNorm weight gradients)
except two float-atomic reductions: the embedding-table gradient scatter (``nd_embedding_bwd``) and
the cross-entropy loss sum.  ``set_deterministic(True)`` swaps them for a stable-argsort + per-run
segment sum (``nd_embedding_bwd_sorted``) and per-row loss values summed by one ordered reduction.
Cost: one device sort of the micro-batch's token ids and a second pass over the embedding grads
(tens of microseconds at 64k tokens)."""
_STATE = {"on": False}


def set_deterministic(enabled: bool) -> None:
    _STATE["on"] = bool(enabled)


def deterministic() -> bool:
    return _STATE["on"]
