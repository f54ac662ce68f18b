"""Cosine-with-warmup LR multiplier, host side.

Same curve as HF ``get_cosine_schedule_with_warmup`` that the reference uses
(REF/nanodiloco/diloco/diloco.py:20): linear warmup from 0, then half-cosine to 0.  Like HF
the multiplier at step 0 is 0 (first inner step runs at lr=0) and the curve keeps
its cosine shape past ``total_steps`` (our trainer stops at ``total_steps`` so that never shows).
The value is a plain Python float passed to the fused optimizer kernel as an argument: no
device tensor, no host sync.
"""
import math


def cosine_with_warmup(step: int, warmup_steps: int, total_steps: int, num_cycles: float = 0.5) -> float:
    if step < warmup_steps:
        return float(step) / float(max(1, warmup_steps))
    progress = float(step - warmup_steps) / float(max(1, total_steps - warmup_steps))
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))


class CosineWarmupSchedule:
    def __init__(self, base_lr: float, warmup_steps: int, total_steps: int):
        self.base_lr = base_lr
        self.warmup_steps = warmup_steps
        self.total_steps = total_steps
        self.step_count = 0

    def lr(self) -> float:
        return self.base_lr * cosine_with_warmup(self.step_count, self.warmup_steps, self.total_steps)

    def step(self):
        self.step_count += 1

    def state_dict(self):
        return {"step_count": self.step_count}

    def load_state_dict(self, d):
        self.step_count = int(d["step_count"])
