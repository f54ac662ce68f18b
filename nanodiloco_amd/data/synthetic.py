"""Synthetic token stream (BASELINE.json: "synthetic data / random-init weights").

Infinite, packed (no padding), uniform over the vocabulary, generated directly on the device by a
per-rank generator: zero host work and zero H2D traffic in the training loop.  Each rank draws from
its own seeded stream (the reference shards a real dataset per rank, REF/nanodiloco/main.py:77).
"""
from __future__ import annotations

import torch

from ..utils.seed import rank_seed


class SyntheticTokens:
    def __init__(self, vocab_size: int, seq_len: int, batch_size: int, seed: int = 1337, rank: int = 0,
                 device="cpu"):
        self.vocab_size = vocab_size
        self.seq_len = seq_len
        self.batch_size = batch_size
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(rank_seed(seed, rank, 1))
        self.samples_drawn = 0

    def __iter__(self):
        return self

    def __next__(self):
        ids = torch.randint(0, self.vocab_size, (self.batch_size, self.seq_len), device=self.device,
                            generator=self.gen)
        self.samples_drawn += self.batch_size
        return {"input_ids": ids, "labels": ids}

    def state_dict(self):
        return {"samples_drawn": self.samples_drawn, "gen_state": self.gen.get_state()}

    def load_state_dict(self, d):
        self.samples_drawn = int(d["samples_drawn"])
        self.gen.set_state(d["gen_state"])
