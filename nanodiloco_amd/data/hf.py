"""HF-datasets path, capability parity with the reference pipeline
(REF/nanodiloco/training_utils/utils.py:45-60, REF/nanodiloco/main.py:75-96):

* ``load_from_disk(dataset_path)`` with ``HF_DATASETS_OFFLINE=1``, batched tokenisation truncated to
  ``seq_length`` (the reference hard-codes 1024 -- SURVEY.md Q5; we honour ``--seq-length``),
  ``text``/``timestamp``/``url`` columns dropped, ``train`` split;
* contiguous per-rank shard (``split_dataset_by_node``);
* collate = pad to the longest sequence rounded up to a multiple of 8, ``labels = input_ids``.
  Pads are masked to -100 (the reference leaves them in the loss, Q5; ``mask_pad_labels=False``
  reproduces that);
* ``DataLoader(batch_size=per_device_batch_size, shuffle=True, drop_last=True)``.

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
        if mask_pad_labels and "attention_mask" in padded:
            labels[padded["attention_mask"] == 0] = -100
        padded["labels"] = labels
        return dict(padded)

    return collate


def make_hf_loader(dataset_path: str, tokenizer_name: str, seq_length: int, per_device_batch_size: int,
                   world_size: int, rank: int, seed: int, mask_pad_labels: bool = True):
    import torch
    from datasets.distributed import split_dataset_by_node
    from torch.utils.data import DataLoader

    tok = get_tokenizer(tokenizer_name)
    ds = get_tokenized_dataset(dataset_path, tok, seq_length)
    shard = split_dataset_by_node(ds, world_size=world_size, rank=rank)
    g = torch.Generator()
    g.manual_seed(seed)
    return DataLoader(shard, batch_size=per_device_batch_size, collate_fn=make_collate(tok, seq_length, mask_pad_labels),
                      drop_last=True, shuffle=True, generator=g)
