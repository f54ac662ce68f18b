"""Reference data path (C10-C12): load_from_disk + tokenize + split_dataset_by_node + pad collate,
with a local tokenizer built offline (no hub access)."""
import os

import pytest
import torch

datasets = pytest.importorskip("datasets")
tokenizers = pytest.importorskip("tokenizers")
transformers = pytest.importorskip("transformers")


def _tokenizer(tmp_path):
    from tokenizers import Tokenizer, models, pre_tokenizers
    vocab = {"<unk>": 0, "<s>": 1, "</s>": 2}
    for w in "the quick brown fox jumps over lazy dog a b c hello world".split():
        vocab[w] = len(vocab)
    tk = Tokenizer(models.WordLevel(vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.Whitespace()
    fast = transformers.PreTrainedTokenizerFast(tokenizer_object=tk, bos_token="<s>", eos_token="</s>",
                                                unk_token="<unk>", padding_side="left")
    d = tmp_path / "tok"
    fast.save_pretrained(str(d))
    return str(d)


def _dataset(tmp_path):
    texts = ["the quick brown fox", "jumps over the lazy dog", "hello world", "a b c a b c a b c",
             "the dog", "hello", "fox fox fox fox fox fox fox", "world world"] * 4
    ds = datasets.DatasetDict({"train": datasets.Dataset.from_dict(
        {"text": texts, "timestamp": ["t"] * len(texts), "url": ["u"] * len(texts)})})
    p = tmp_path / "ds"
    ds.save_to_disk(str(p))
    return str(p)


def test_hf_loader_pads_masks_and_shards(tmp_path):
    from nanodiloco_amd.data.hf import make_hf_loader
    tok, ds = _tokenizer(tmp_path), _dataset(tmp_path)
    seen = []
    for rank in range(2):
        dl = make_hf_loader(ds, tok, seq_length=16, per_device_batch_size=4, world_size=2, rank=rank, seed=0)
        n = 0
        assert len(dl) == 4
        for _ in range(len(dl)):
            b = next(dl)
            ids, lab, am = b["input_ids"], b["labels"], b["attention_mask"]
            assert ids.shape[1] % 8 == 0 and ids.shape[0] == 4
            assert torch.equal(lab[am == 1], ids[am == 1])
            assert (lab[am == 0] == -100).all()                  # pads masked (reference leaves them in, Q5)
            n += 1
        seen.append(n)
    assert seen == [4, 4]  # 16 docs per rank, contiguous shards, drop_last


def test_trainer_hf_path_runs(tmp_path):
    from nanodiloco_amd.trainer import TrainArgs, Trainer
    tok, ds = _tokenizer(tmp_path), _dataset(tmp_path)
    cfg = tmp_path / "m.json"
    cfg.write_text('{"hidden_size": 32, "intermediate_size": 64, "num_attention_heads": 2, '
                   '"num_hidden_layers": 1, "vocab_size": 32}')
    out = Trainer(TrainArgs(batch_size=4, per_device_batch_size=2, seq_length=16, warmup_steps=1, total_steps=4,
                            inner_steps=2, dataset_path=ds, tokenizer=tok, llama_config_file=str(cfg), wandb="off",
                            device="cpu", data="hf")).train()
    assert out["steps"] == 4 and out["outer_steps"] == 2


def test_hf_loader_resumes_from_cursor(tmp_path):
    from nanodiloco_amd.data.hf import make_hf_loader
    tok, ds = _tokenizer(tmp_path), _dataset(tmp_path)
    mk = lambda: make_hf_loader(ds, tok, seq_length=16, per_device_batch_size=4, world_size=2, rank=1, seed=3)
    a = mk()
    for _ in range(6):  # crosses the epoch boundary (4 batches per epoch)
        next(a)
    st = a.state_dict()
    assert st == {"epoch": 1, "batch": 2}
    b = mk()
    b.load_state_dict(st)
    for _ in range(5):
        x, y = next(a), next(b)
        assert torch.equal(x["input_ids"], y["input_ids"]) and torch.equal(x["labels"], y["labels"])
