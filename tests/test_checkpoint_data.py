"""Checkpoint format (HF-loadable + resumable) and the native memmap token loader."""
import json
import os

import numpy as np
import pytest
import torch

from nanodiloco_amd.config import LlamaConfig
from nanodiloco_amd.models import LlamaForCausalLM
from nanodiloco_amd.optim import FlatAdamW, FlatOuterNesterov
from nanodiloco_amd.parallel.diloco import Diloco
from nanodiloco_amd.parallel.dist import DistEnv
from nanodiloco_amd.utils.checkpoint import load_checkpoint, save_checkpoint

CFG = dict(hidden_size=32, intermediate_size=64, num_attention_heads=2, num_hidden_layers=2, vocab_size=60,
           rms_norm_eps=1e-5)


def _mk(seed=0):
    m = LlamaForCausalLM(LlamaConfig.from_dict(CFG)).init_weights(seed)
    d = Diloco(m, FlatAdamW(m.store, lr=1e-3), FlatOuterNesterov(m.store), 2, 8, 4, env=DistEnv())
    return m, d


def _train(m, d, steps, g):
    for s in range(steps):
        ids = torch.randint(0, 60, (2, 16), generator=g)
        m(ids, labels=ids).loss.backward()
        d.inner_step()
        if (s + 1) % 4 == 0:
            d.outer_step()


def test_checkpoint_roundtrip_and_resume(tmp_path):
    m, d = _mk()
    g = torch.Generator().manual_seed(0)
    _train(m, d, 4, g)
    save_checkpoint(str(tmp_path), m, d, DistEnv(), step=4)
    assert {"config.json", "model.safetensors", "diloco_state.safetensors", "rank0.safetensors",
            "trainer_state.json"} <= set(os.listdir(tmp_path))
    # continue original
    g1 = torch.Generator().manual_seed(1)
    _train(m, d, 4, g1)
    # resume a fresh one from the checkpoint with the same data
    m2, d2 = _mk(seed=99)
    st = load_checkpoint(str(tmp_path), m2, d2, DistEnv())
    assert st["step"] == 4
    g2 = torch.Generator().manual_seed(1)
    _train(m2, d2, 4, g2)
    assert torch.allclose(m.store.master, m2.store.master, atol=1e-6)
    assert d.outer_step_count == d2.outer_step_count == 2


def test_checkpoint_refuses_other_topology(tmp_path):
    """A resume with another world size / --inner-dp / model would drop workers' AdamW state or
    mis-shard the outer momentum: load_checkpoint refuses it."""
    m, d = _mk()
    save_checkpoint(str(tmp_path), m, d, DistEnv(), step=0)
    st = json.load(open(tmp_path / "trainer_state.json"))
    assert (st["world_size"], st["inner_dp"], st["flat_numel"], st["pending_outer"]) == (1, 1, m.store.numel, False)
    for key, val in (("world_size", 2), ("inner_dp", 2), ("flat_numel", m.store.numel + 64)):
        bad = dict(st, **{key: val})
        json.dump(bad, open(tmp_path / "trainer_state.json", "w"))
        m2, d2 = _mk(1)
        with pytest.raises(ValueError, match=key):
            load_checkpoint(str(tmp_path), m2, d2, DistEnv())
    json.dump(st, open(tmp_path / "trainer_state.json", "w"))
    os.remove(tmp_path / "rank0.safetensors")
    with pytest.raises(FileNotFoundError):
        load_checkpoint(str(tmp_path), *_mk(1), DistEnv())


def test_checkpoint_keeps_overlapped_outer_step_pending(tmp_path):
    """--overlap-outer: a checkpoint at the boundary saves the outer step as pending; resumed, the
    next inner step applies it -- same weights as the run that never stopped."""
    def mk(seed):
        m = LlamaForCausalLM(LlamaConfig.from_dict(CFG)).init_weights(seed)
        return m, Diloco(m, FlatAdamW(m.store, lr=1e-3), FlatOuterNesterov(m.store), 2, 8, 4, env=DistEnv(),
                         overlap=True)
    m, d = mk(0)
    _train(m, d, 4, torch.Generator().manual_seed(0))
    assert d._pending is not None
    save_checkpoint(str(tmp_path), m, d, DistEnv(), step=4)
    assert json.load(open(tmp_path / "trainer_state.json"))["pending_outer"] is True
    assert d._pending is not None  # saving did not apply it
    _train(m, d, 4, torch.Generator().manual_seed(1))
    m2, d2 = mk(99)
    load_checkpoint(str(tmp_path), m2, d2, DistEnv())
    assert d2._pending is not None
    _train(m2, d2, 4, torch.Generator().manual_seed(1))
    d.finalize(), d2.finalize()
    assert torch.equal(m.store.master, m2.store.master) and torch.equal(d.sync, d2.sync)


def test_checkpoint_loads_into_hf(tmp_path):
    transformers = pytest.importorskip("transformers")
    m, d = _mk(3)
    save_checkpoint(str(tmp_path), m, d, DistEnv(), step=0)
    hf = transformers.LlamaForCausalLM.from_pretrained(str(tmp_path), attn_implementation="eager").float()
    ids = torch.randint(0, 60, (2, 12))
    assert torch.allclose(hf(input_ids=ids).logits, m(ids).logits, atol=1e-5)
    cfg = json.load(open(tmp_path / "config.json"))
    assert cfg["architectures"] == ["LlamaForCausalLM"]


@pytest.fixture(scope="module")
def runtime_lib():
    from nanodiloco_amd.csrc.build import build
    try:
        build()
    except FileNotFoundError:
        pytest.skip("no hipcc")
    from nanodiloco_amd.data.memmap import runtime_lib as rl
    return rl()


def test_memmap_loader_disjoint_deterministic(tmp_path, runtime_lib):
    from nanodiloco_amd.data.memmap import MemmapTokens, write_token_shard
    T = 16
    toks = np.arange(40 * T) % 30000
    write_token_shard(str(tmp_path / "a.bin"), toks[: 25 * T])
    write_token_shard(str(tmp_path / "b.bin"), toks[25 * T:])
    paths = [str(tmp_path / "a.bin"), str(tmp_path / "b.bin")]
    seen = []
    for r in range(2):
        L = MemmapTokens(paths, T, 4, rank=r, world_size=2, seed=5)
        assert L.windows_per_rank == 20
        rows = torch.cat([next(L)["input_ids"] for _ in range(5)])  # one epoch = 20 windows
        starts = set((rows[:, 0] // T).tolist())
        assert len(starts) == 20
        # the two workers read disjoint halves of the global stream (positions r, r + 2, r + 4, ...)
        assert starts == {L.window_of(k) for k in range(20)}
        assert torch.equal(rows[:, 1:] - rows[:, :-1], torch.ones_like(rows[:, 1:]))  # contiguous windows
        seen.append(starts)
        L.close()
    assert not (seen[0] & seen[1])
    # determinism + seek/resume
    A = MemmapTokens(paths, T, 4, rank=0, world_size=2, seed=5)
    first = [next(A)["input_ids"].clone() for _ in range(7)]
    B = MemmapTokens(paths, T, 4, rank=0, world_size=2, seed=5)
    for _ in range(3):
        next(B)
    stt = B.state_dict()
    C = MemmapTokens(paths, T, 4, rank=0, world_size=2, seed=5)
    C.load_state_dict(stt)
    for i in range(3, 7):
        assert torch.equal(next(C)["input_ids"], first[i])


def test_memmap_elastic_resume_repeats_and_skips_nothing(tmp_path, runtime_lib):
    """--elastic-resume on another worker count.  Two workers read 3 batches each of epoch 0, then
    the job resumes on 3 workers from rank 0's state (every worker, survivor or new, gets the same state):
    until epoch 0 is done no window is read twice and every window is read once."""
    from nanodiloco_amd.data.memmap import MemmapTokens, write_token_shard
    T, B, G = 8, 2, 60
    write_token_shard(str(tmp_path / "a.bin"), np.arange(G * T) % 30000)
    paths = [str(tmp_path / "a.bin")]

    def windows(L, n):
        return [int(w) for w in (torch.cat([next(L)["input_ids"] for _ in range(n)])[:, 0] // T).tolist()]

    old = [MemmapTokens(paths, T, B, rank=r, world_size=2, seed=3) for r in range(2)]
    read = sum((windows(L, 3) for L in old), [])  # 2 workers x 3 batches x 2 = 12 windows
    st = old[0].state_dict()
    assert st == {"cursor": 6, "base": 0, "world": 2}
    new = [MemmapTokens(paths, T, B, rank=r, world_size=3, seed=3) for r in range(3)]
    for L in new:
        L.load_state_dict(st, resized=True)
        assert L.state_dict() == {"cursor": 0, "base": 12, "world": 3}
    read += sum((windows(L, 8) for L in new), [])  # 3 x 8 x 2 = 48 more: epoch 0 complete
    assert len(read) == G and len(set(read)) == G  # nothing repeated, nothing skipped
    # a normal (same-count) resume of a resized stream continues it exactly
    nxt = windows(new[1], 2)
    again = MemmapTokens(paths, T, B, rank=1, world_size=3, seed=3)
    again.load_state_dict({"cursor": 16, "base": 12, "world": 3})
    assert windows(again, 2) == nxt
    for L in old + new + [again]:
        L.close()
