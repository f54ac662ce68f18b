"""HF-datasets path, capability parity with the reference pipeline
(REF/nanodiloco/training_utils/utils.py:45-60, REF/nanodiloco/main.py:75-96):

* ``load_from_disk(dataset_path)`` with ``HF_DATASETS_OFFLINE=1``, batched tokenisation truncated to
  ``seq_length`` (the reference hard-codes 1024 -- SURVEY.md Q5; we honour ``--seq-length``),
  ``text``/``timestamp``/``url`` columns dropped, ``train`` split;
* contiguous per-rank shard (``split_dataset_by_node``);
* collate = pad to the longest sequence rounded up to a multiple of 8, ``labels = input_ids``.
  Pads are masked to -100 (the reference leaves them in the loss, Q5; ``mask_pad_labels=False``
  reproduces that);
* ``DataLoader(batch_size=per_device_batch_size, shuffle=True, drop_last=True)`` semantics, as a
  resumable batch iterator (:class:`HFBatches`: the cursor is checkpointed).

Tokeniser: ``AutoTokenizer.from_pretrained(name)`` with ``pad_token = "</s>"`` (reference default
``huggyllama/llama-7b``); it must be available locally (no network on MI355X boxes).  For
production runs prefer the pre-tokenised memmap path (``data/memmap.py``) which needs no tokenizer
at train time.
"""
from __future__ import annotations

import os


def get_tokenizer(name: str = "huggyllama/llama-7b"):
    from transformers import AutoTokenizer

    tok = AutoTokenizer.from_pretrained(name)
    tok.pad_token = "</s>"
    return tok


def get_tokenized_dataset(dataset_path: str, tokenizer, seq_length: int = 1024, num_proc: int = 1):
    os.environ["HF_DATASETS_OFFLINE"] = "1"
    from datasets import load_from_disk

    ds = load_from_disk(dataset_path)

    def tok_fn(batch):
        return tokenizer(batch["text"], truncation=True, max_length=seq_length)

    cols = [c for c in ("text", "timestamp", "url") if c in ds["train"].column_names]
    ds = ds.map(tok_fn, batched=True, remove_columns=cols, num_proc=num_proc)
    return ds["train"]


def make_collate(tokenizer, seq_length: int, mask_pad_labels: bool = True):
    def collate(batch):
        padded = tokenizer.pad(batch, padding="longest", max_length=seq_length, pad_to_multiple_of=8,
                               return_tensors="pt")
        labels = padded["input_ids"].clone()
        if "attention_mask" in padded:
            # the attention kernels take one key start per sequence (left / right padding only): a mask
            # with a hole would silently attend with the wrong mask, so reject it here, on the host copy
            # (no device sync)
            from ..ops.attention import check_padding
            check_padding(padded["attention_mask"])
        if mask_pad_labels and "attention_mask" in padded:
            labels[padded["attention_mask"] == 0] = -100
        padded["labels"] = labels
        return dict(padded)

    return collate


class HFBatches:
    """Resumable replacement for ``DataLoader(shard, batch_size, shuffle=True, drop_last=True,
    collate_fn)`` (REF/nanodiloco/main.py:90-96; ``num_workers=0`` there too).

    Epoch ``e`` visits the shard in the permutation drawn from ``torch.Generator().manual_seed(
    seed + e)`` (same on every rank, like the reference's same-seed shuffle), in full batches only.
    The cursor ``(epoch, batch)`` is the whole state, so a resumed run continues with exactly the
    batch an uninterrupted run would have drawn.  Iterating past the last full batch of an epoch
    moves to the next epoch (the trainer is bounded by ``total_steps``, not by epochs)."""

    def __init__(self, shard, batch_size: int, collate, seed: int):
        if len(shard) < batch_size:
            raise ValueError(f"dataset shard has {len(shard)} rows < per-device batch {batch_size}")
        self.shard, self.batch_size, self.collate, self.seed = shard, batch_size, collate, int(seed)
        self.epoch, self.batch = 0, 0
        self._perm = None

    @property
    def batches_per_epoch(self) -> int:
        return len(self.shard) // self.batch_size

    def _order(self):
        if self._perm is None:
            import torch
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            self._perm = torch.randperm(len(self.shard), generator=g).tolist()
        return self._perm

    def __iter__(self):
        return self

    def __len__(self):
        return self.batches_per_epoch

    def __next__(self):
        if self.batch >= self.batches_per_epoch:
            self.epoch, self.batch, self._perm = self.epoch + 1, 0, None
        idx = self._order()[self.batch * self.batch_size:(self.batch + 1) * self.batch_size]
        self.batch += 1
        return self.collate([self.shard[i] for i in idx])

    def state_dict(self):
        return {"epoch": self.epoch, "batch": self.batch}

    def load_state_dict(self, d):
        self.epoch, self.batch, self._perm = int(d["epoch"]), int(d["batch"]), None


def make_hf_loader(dataset_path: str, tokenizer_name: str, seq_length: int, per_device_batch_size: int,
                   world_size: int, rank: int, seed: int, mask_pad_labels: bool = True) -> HFBatches:
    from datasets.distributed import split_dataset_by_node

    tok = get_tokenizer(tokenizer_name)
    ds = get_tokenized_dataset(dataset_path, tok, seq_length)
    shard = split_dataset_by_node(ds, world_size=world_size, rank=rank)
    return HFBatches(shard, per_device_batch_size, make_collate(tok, seq_length, mask_pad_labels), seed)
