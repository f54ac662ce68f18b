"""Data sources: synthetic on-device tokens, native memmap shards, HF datasets (reference path)."""
from .synthetic import SyntheticTokens


def build_data(kind: str, *, vocab_size: int, seq_len: int, batch_size: int, seed: int, rank: int,
               world_size: int, device, dataset_path: str = None, tokenizer: str = "huggyllama/llama-7b",
               mask_pad_labels: bool = True):
    if kind == "synthetic":
        return SyntheticTokens(vocab_size, seq_len, batch_size, seed, rank, device)
    if kind == "memmap":
        import glob
        import os

        from .memmap import MemmapTokens
        paths = sorted(glob.glob(os.path.join(dataset_path, "*.bin"))) if os.path.isdir(dataset_path) \
            else sorted(glob.glob(dataset_path))
        if not paths:
            raise FileNotFoundError(f"no token shards at {dataset_path}")
        return MemmapTokens(paths, seq_len, batch_size, vocab_size, seed, rank, world_size, device=device)
    if kind == "hf":
        from .hf import make_hf_loader
        return _DeviceIter(make_hf_loader(dataset_path, tokenizer, seq_len, batch_size, world_size, rank, seed,
                                          mask_pad_labels), device)
    raise ValueError(f"unknown data source {kind}")


class _DeviceIter:
    """Moves host batches to the device; forwards the loader's resumable cursor."""

    def __init__(self, loader, device):
        self.loader, self.device = loader, device

    def __iter__(self):
        return self

    def __next__(self):
        b = next(self.loader)
        return {k: v.to(self.device, non_blocking=True) for k, v in b.items()}

    def state_dict(self):
        return self.loader.state_dict()

    def load_state_dict(self, d, resized: bool = False):
        if resized:
            # HFBatches: each rank reads a CONTIGUOUS shard of the dataset (split_dataset_by_node, the
            # reference's sharding); another worker count re-cuts every shard, so no cursor maps onto the
            # new layout without repeating or skipping examples
            raise RuntimeError("--elastic-resume with --data hf cannot keep the data stream exact (the contiguous "
                               "per-rank shards move with the worker count); use --data memmap (pre-tokenised "
                               "shards, scripts/pretokenize.py), whose global stream resumes exactly on any count")
        self.loader.load_state_dict(d)


__all__ = ["SyntheticTokens", "build_data"]
