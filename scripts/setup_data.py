#!/usr/bin/env python3
"""Materialise a training dataset on local disk -- the capability equivalent of the reference's
``materialize_c4_tiny`` (REF/scripts/setup_data_volume.py:6-61), without network access:

  * ``--from-hf NAME [--config en]``  load from the local HF cache (HF_DATASETS_OFFLINE=1) and
    ``save_to_disk`` to ``<out>/datasets/<NAME>/<config>/save_to_disk`` (the path layout the reference
    uses), then write ``manifest.json``;
  * ``--from-text FILE...``           build the same ``{"train": {"text", "timestamp", "url"}}`` layout
    from local text / JSONL files (one document per line, or a ``text`` field);
  * ``--pretokenize --tokenizer T``   additionally write memmap token shards (scripts/pretokenize.py)
    for ``--data memmap``.
"""
import argparse
import json
import os
import subprocess
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="/vol")
    ap.add_argument("--from-hf")
    ap.add_argument("--config", default="en")
    ap.add_argument("--from-text", nargs="*")
    ap.add_argument("--pretokenize", action="store_true")
    ap.add_argument("--tokenizer", default="huggyllama/llama-7b")
    a = ap.parse_args()
    os.environ["HF_DATASETS_OFFLINE"] = "1"
    import datasets

    if a.from_hf:
        ds = datasets.load_dataset(a.from_hf, a.config)
        dest = os.path.join(a.out, "datasets", a.from_hf, a.config, "save_to_disk")
    elif a.from_text:
        texts = []
        for p in a.from_text:
            with open(p, encoding="utf-8") as f:
                for line in f:
                    line = line.strip()
                    if not line:
                        continue
                    if line.startswith("{"):
                        line = json.loads(line).get("text", "")
                    texts.append(line)
        ds = datasets.DatasetDict({"train": datasets.Dataset.from_dict(
            {"text": texts, "timestamp": [""] * len(texts), "url": [""] * len(texts)})})
        dest = os.path.join(a.out, "datasets", "local", "text", "save_to_disk")
    else:
        ap.error("need --from-hf or --from-text")
    os.makedirs(dest, exist_ok=True)
    ds.save_to_disk(dest)
    manifest = {"path": dest, "splits": {k: len(v) for k, v in ds.items()}, "columns": ds["train"].column_names}
    with open(os.path.join(os.path.dirname(dest), "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=2)
    print(json.dumps(manifest))
    if a.pretokenize:
        tok_dir = os.path.join(os.path.dirname(dest), "tokens")
        rc = subprocess.call([sys.executable, os.path.join(os.path.dirname(__file__), "pretokenize.py"),
                              "--dataset-path", dest, "--tokenizer", a.tokenizer, "--out-dir", tok_dir])
        sys.exit(rc)


if __name__ == "__main__":
    main()
