"""Seeding (REF/nanodiloco/training_utils/utils.py:11-15).

Every rank uses the same seed, exactly like the reference, so the model init is identical on
all workers before the (flat) broadcast.  Data streams are decorrelated per rank separately
(:func:`rank_seed`).
"""
import random

import numpy as np
import torch


def set_seed_all(seed: int = 42) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def rank_seed(seed: int, rank: int, stream: int = 0) -> int:
    """Deterministic per-rank / per-stream seed (splitmix-style mixing, fits in int63)."""
    x = (seed * 0x9E3779B97F4A7C15 + rank * 0xBF58476D1CE4E5B9 + stream * 0x94D049BB133111EB) & ((1 << 64) - 1)
    x ^= x >> 31
    x = (x * 0xD6E8FEB86659FD93) & ((1 << 64) - 1)
    x ^= x >> 32
    return x & ((1 << 63) - 1)
