#!/usr/bin/env python3
"""Pre-tokenise a corpus into flat token shards for the native memmap loader (``--data memmap``).

The reference tokenises c4-tiny on every rank at start-up (REF/nanodiloco/training_utils/utils.py:45-55);
here that happens once, offline:

  python scripts/pretokenize.py --dataset-path /path/to/save_to_disk --tokenizer /path/to/tokenizer \
      --out-dir /data/c4tiny_tokens --shard-tokens 100000000

Inputs: an HF ``save_to_disk`` dataset (``--dataset-path``, column ``text``) or plain ``--text-files``.
Each document is tokenised (BOS added by the tokenizer, EOS appended here) and concatenated; shards
are little-endian uint16 (vocab <= 65535) or uint32.  A ``manifest.json`` records counts.
Everything stays local: the tokenizer must be a local path or already cached.
"""
import argparse
import json
import os

import numpy as np


def iter_texts(a):
    if a.text_files:
        for p in a.text_files:
            with open(p, encoding="utf-8") as f:
                for line in f:
                    line = line.strip()
                    if line:
                        yield line
        return
    os.environ["HF_DATASETS_OFFLINE"] = "1"
    from datasets import load_from_disk

    ds = load_from_disk(a.dataset_path)
    split = ds[a.split] if hasattr(ds, "keys") else ds
    for row in split:
        yield row[a.column]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset-path")
    ap.add_argument("--text-files", nargs="*")
    ap.add_argument("--split", default="train")
    ap.add_argument("--column", default="text")
    ap.add_argument("--tokenizer", default="huggyllama/llama-7b")
    ap.add_argument("--out-dir", required=True)
    ap.add_argument("--shard-tokens", type=int, default=100_000_000)
    ap.add_argument("--batch", type=int, default=1000)
    a = ap.parse_args()
    from transformers import AutoTokenizer

    tok = AutoTokenizer.from_pretrained(a.tokenizer)
    dt = np.uint16 if len(tok) <= 65535 else np.uint32
    eos = tok.eos_token_id
    os.makedirs(a.out_dir, exist_ok=True)
    buf, shards, total, docs = [], [], 0, 0

    def flush(final=False):
        nonlocal buf
        while len(buf) >= a.shard_tokens or (final and buf):
            chunk, buf = buf[: a.shard_tokens], buf[a.shard_tokens:]
            path = os.path.join(a.out_dir, f"shard_{len(shards):05d}.bin")
            np.asarray(chunk, dtype=dt).tofile(path)
            shards.append({"path": os.path.basename(path), "tokens": len(chunk)})

    batch = []
    for text in iter_texts(a):
        batch.append(text)
        if len(batch) == a.batch:
            for ids in tok(batch)["input_ids"]:
                buf.extend(ids + [eos])
                total += len(ids) + 1
                docs += 1
            batch = []
            flush()
    if batch:
        for ids in tok(batch)["input_ids"]:
            buf.extend(ids + [eos])
            total += len(ids) + 1
            docs += 1
    flush(final=True)
    with open(os.path.join(a.out_dir, "manifest.json"), "w") as f:
        json.dump({"tokenizer": a.tokenizer, "dtype": np.dtype(dt).name, "vocab_size": len(tok), "documents": docs,
                   "tokens": total, "shards": shards}, f, indent=2)
    print(f"wrote {len(shards)} shards, {total} tokens, {docs} documents -> {a.out_dir}")


if __name__ == "__main__":
    main()
