"""Pre-tokenised memmap token stream backed by the native C++ loader
(``nanodiloco_amd/csrc/runtime/token_loader.cpp`` -> ``_lib/libnd_runtime.so``).

Shard format: flat little-endian ``uint16`` (vocab <= 65535) or ``uint32`` token ids, documents
concatenated (separate them with EOS when writing).  ``write_token_shard`` / ``scripts/pretokenize.py``
produce it.  Batches are ``int64 [batch, seq_len]`` assembled by a background C++ thread into a
ring of pinned host buffers and copied to the device with a non-blocking H2D copy.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
RUNTIME_LIB = os.path.join(os.path.dirname(_HERE), "_lib", "libnd_runtime.so")
_rt = None


def runtime_lib():
    global _rt
    if _rt is None:
        if not os.path.exists(RUNTIME_LIB):
            raise FileNotFoundError(f"{RUNTIME_LIB} missing: run `python -m nanodiloco_amd.csrc.build`")
        L = ctypes.CDLL(RUNTIME_LIB)
        P, I, I64, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64
        L.nd_loader_create.argtypes = [ctypes.c_char_p, I, I64, I64, U64, I, I, I, I, ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.c_char_p, I]
        L.nd_loader_create.restype = P
        L.nd_loader_next.argtypes = [P]
        L.nd_loader_next.restype = I
        L.nd_loader_release.argtypes = [P, I]
        L.nd_loader_release.restype = None
        L.nd_loader_cursor.argtypes = [P]
        L.nd_loader_cursor.restype = I64
        L.nd_loader_seek.argtypes = [P, I64]
        L.nd_loader_seek.restype = None
        L.nd_loader_destroy.argtypes = [P]
        L.nd_loader_destroy.restype = None
        L.nd_loader_windows_per_rank.argtypes = [P]
        L.nd_loader_windows_per_rank.restype = I64
        L.nd_loader_total_windows.argtypes = [P]
        L.nd_loader_total_windows.restype = I64
        L.nd_loader_base.argtypes = [P]
        L.nd_loader_base.restype = I64
        L.nd_loader_set_base.argtypes = [P, I64, I64]
        L.nd_loader_set_base.restype = None
        L.nd_loader_window_of.argtypes = [P, I64]
        L.nd_loader_window_of.restype = I64
        _rt = L
    return _rt


def write_token_shard(path: str, tokens, vocab_size: int = 32000):
    dt = np.uint16 if vocab_size <= 65535 else np.uint32
    np.asarray(tokens, dtype=dt).tofile(path)


class MemmapTokens:
    def __init__(self, paths: Sequence[str], seq_len: int, batch_size: int, vocab_size: int = 32000,
                 seed: int = 1337, rank: int = 0, world_size: int = 1, shuffle: bool = True, prefetch: int = 4,
                 device="cpu"):
        self.paths: List[str] = [os.path.abspath(p) for p in paths]
        self.seq_len, self.batch_size = seq_len, batch_size
        self.device = torch.device(device)
        self.token_bytes = 2 if vocab_size <= 65535 else 4
        pin = self.device.type == "cuda"
        self.slots = [torch.empty(batch_size, seq_len, dtype=torch.int64, pin_memory=pin) for _ in range(prefetch)]
        arr = (ctypes.c_void_p * prefetch)(*[s.data_ptr() for s in self.slots])
        err = ctypes.create_string_buffer(512)
        L = runtime_lib()
        self.h = L.nd_loader_create("\n".join(self.paths).encode(), self.token_bytes, seq_len, batch_size, seed,
                                    rank, world_size, 1 if shuffle else 0, prefetch, arr, err, 512)
        if not self.h:
            raise RuntimeError(f"token loader: {err.value.decode()}")
        self.world_size = world_size
        self._pending = []

    @property
    def windows_per_rank(self) -> int:
        return runtime_lib().nd_loader_windows_per_rank(self.h)

    @property
    def total_windows(self) -> int:
        return runtime_lib().nd_loader_total_windows(self.h)

    def window_of(self, sample: int) -> int:
        """Global window index this rank's sample ``sample`` (counted from the stream base) reads."""
        return runtime_lib().nd_loader_window_of(self.h, int(sample))

    def __iter__(self):
        return self

    def _drain(self):
        L = runtime_lib()
        for slot, ev in self._pending:
            if ev is not None:
                ev.synchronize()
            L.nd_loader_release(self.h, slot)
        self._pending = []

    def __next__(self):
        L = runtime_lib()
        self._drain()
        slot = L.nd_loader_next(self.h)
        host = self.slots[slot]
        if self.device.type == "cuda":
            ids = torch.empty_like(host, device=self.device)
            ids.copy_(host, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._pending.append((slot, ev))
        else:
            ids = host.clone()
            self._pending.append((slot, None))
        return {"input_ids": ids, "labels": ids}

    def state_dict(self):
        L = runtime_lib()
        return {"cursor": L.nd_loader_cursor(self.h), "base": L.nd_loader_base(self.h), "world": self.world_size}

    def load_state_dict(self, d, resized: bool = False):
        """``resized`` (``--elastic-resume`` onto a different number of workers): ``d`` is any worker's state
        (they advance in lockstep); this rank restarts the global stream at the position the old workers had
        reached together (base + cursor * old world), so no window is repeated or skipped across the resize."""
        self._drain()
        L = runtime_lib()
        cursor, base = int(d.get("cursor", 0)), int(d.get("base", 0))
        world = int(d.get("world", self.world_size))
        if resized or world != self.world_size:
            L.nd_loader_set_base(self.h, base + cursor * world, 0)
        else:
            L.nd_loader_set_base(self.h, base, cursor)

    def close(self):
        if getattr(self, "h", None):
            self._drain()
            runtime_lib().nd_loader_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
