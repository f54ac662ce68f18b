"""T0: config schema, CLI flag parity, run naming, LR schedule."""
import json
import os
import re
from datetime import datetime

import pytest

from nanodiloco_amd.config import LlamaConfig, default_llama_config, default_run_config, resolve_llama_config
from nanodiloco_amd.main import build_parser, parse_args
from nanodiloco_amd.utils.run_name import create_run_name
from nanodiloco_amd.utils.schedule import CosineWarmupSchedule, cosine_with_warmup

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_FLAGS = {  # REF/nanodiloco/main.py:42-56
    "seed": 1337, "batch_size": 256, "per_device_batch_size": 8, "seq_length": 1024, "warmup_steps": 100,
    "total_steps": 10_000, "inner_steps": 100, "lr": 4e-4, "outer_lr": 0.7, "project": "nano-diloco",
    "dataset_path": "/mnt/hf-c4-tiny/datasets/PrimeIntellect/c4-tiny/en/save_to_disk",
    "llama_config_file": None, "wandb_config_file": None,
}


def test_reference_flags_and_defaults():
    a = parse_args([])
    for k, v in REF_FLAGS.items():
        assert getattr(a, k) == v, k


def test_kebab_case_flags_parse():
    a = parse_args(["--batch-size=128", "--lr=1e-3", "--total-steps=5000", "--per-device-batch-size", "16",
                    "--llama-config-file", "configs/llama_default.json", "--wandb-config-file", "x.json",
                    "--outer-lr", "0.5", "--inner-steps", "50", "--seq-length", "512", "--warmup-steps", "10",
                    "--project", "p", "--dataset-path", "/d", "--seed", "1"])
    assert (a.batch_size, a.lr, a.total_steps, a.per_device_batch_size, a.outer_lr, a.inner_steps) == \
        (128, 1e-3, 5000, 16, 0.5, 50)


def test_reference_json_configs_load_unchanged():
    c = LlamaConfig.from_json(os.path.join(ROOT, "configs", "llama_default.json"))
    assert (c.hidden_size, c.intermediate_size, c.num_attention_heads, c.num_hidden_layers) == (128, 512, 4, 6)
    assert c.vocab_size == 32000 and c.num_key_value_heads == 4 and c.head_dim == 32
    assert c.rms_norm_eps == 1e-5 and c.rope_theta == 10000.0 and not c.tie_word_embeddings
    assert c.num_params() == 9_766_528                      # SURVEY.md §2.3 probe
    assert len(c.param_shapes()) == 57
    large = LlamaConfig.from_json(os.path.join(ROOT, "configs", "llama_large.json"))
    assert large.num_params() == 28_973_312 and len(large.param_shapes()) == 111
    c150 = resolve_llama_config("llama_150m.json")
    assert abs(c150.num_params() - 215.0e6) < 0.5e6
    c1b = resolve_llama_config("llama_1b.json")
    assert abs(c1b.num_params() - 1100.0e6) < 2e6 and c1b.num_key_value_heads == 4


def test_in_code_defaults():
    assert LlamaConfig.from_dict(default_llama_config()).num_params() == 9_766_528
    assert default_run_config() == {"nodes": 1, "location": "local", "backend": "nccl", "measure_comms": True}


def test_unknown_keys_roundtrip_and_hf_json():
    c = LlamaConfig.from_dict({**default_llama_config(), "some_future_key": 3})
    d = c.to_dict()
    assert d["some_future_key"] == 3 and d["architectures"] == ["LlamaForCausalLM"]
    hf = c.to_hf_json()
    assert hf["model_type"] == "llama"
    transformers = pytest.importorskip("transformers")
    hc = transformers.LlamaConfig(**{k: v for k, v in hf.items() if k not in ("some_future_key",)})
    assert hc.hidden_size == 128


def test_transformers_v5_rope_parameters_spelling():
    c = LlamaConfig.from_dict({"hidden_size": 64, "num_attention_heads": 2,
                               "rope_parameters": {"rope_theta": 500000.0, "rope_type": "default"}})
    assert c.rope_theta == 500000.0


def test_run_name_format():
    n = create_run_name("nanodiloco", {"nodes": 2, "location": "modal"}, now=datetime(2026, 3, 4, 5, 6))
    assert re.fullmatch(r"nanodiloco_n2_modal_0304_0506_[0-9a-f]{8}", n), n
    d = create_run_name("nanodiloco", {}, is_debug=True, now=datetime(2026, 3, 4, 5, 6))
    assert re.fullmatch(r"debug_nanodiloco_0304_0506_[0-9a-f]{8}", d), d


def test_cosine_schedule_matches_hf():
    transformers = pytest.importorskip("transformers")
    import torch
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=4e-4)
    s = transformers.get_cosine_schedule_with_warmup(opt, num_warmup_steps=100, num_training_steps=10000)
    ours = CosineWarmupSchedule(4e-4, 100, 10000)
    for step in range(0, 10000, 37):
        while ours.step_count < step:
            ours.step()
            s.step()
        assert abs(opt.param_groups[0]["lr"] - ours.lr()) < 1e-12
    assert cosine_with_warmup(0, 100, 10000) == 0.0  # lr = 0 at the first inner step (Q4)


def test_trainer_asserts_like_reference():
    from nanodiloco_amd.trainer import TrainArgs, Trainer
    with pytest.raises(ValueError):
        Trainer(TrainArgs(batch_size=10, per_device_batch_size=3, device="cpu"))
    with pytest.raises(ValueError):
        Trainer(TrainArgs(total_steps=10, inner_steps=3, device="cpu"))


def test_launcher_fault_tolerant_and_elastic_commands():
    """scripts/launch.py: --fault-tolerant adds restarts + per-outer-step checkpoints + --resume auto; --min-nodes
    switches to an elastic c10d rendezvous (nnodes MIN:MAX) with --elastic-resume."""
    import argparse
    import importlib.util
    spec = importlib.util.spec_from_file_location("launch", os.path.join(ROOT, "scripts", "launch.py"))
    L = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(L)
    base = dict(cmd="main", nnodes=2, node_rank=0, master_addr="10.0.0.1", master_port=29500, nproc_per_node=8,
                max_restarts=None, fault_tolerant=False, min_nodes=0, checkpoint_dir=None, run_id="r", extra=[],
                dry_run=True)
    plain = L.torchrun_cmd(argparse.Namespace(**base), [])
    assert "--max-restarts=0" in plain and "--resume" not in plain and "--node-rank=0" in plain
    ft = L.torchrun_cmd(argparse.Namespace(**{**base, "fault_tolerant": True, "checkpoint_dir": "/ck"}), [])
    assert "--max-restarts=3" in ft and ft[ft.index("--resume") + 1] == "auto" and "/ck" in ft
    el = L.torchrun_cmd(argparse.Namespace(**{**base, "min_nodes": 1}), [])
    assert "--nnodes=1:2" in el and "--rdzv-backend=c10d" in el and "--elastic-resume" in el
    assert "--max-restarts=3" in el and "--node-rank=0" not in el
    from nanodiloco_amd import main as M
    a = M.parse_args(el[el.index("nanodiloco_amd") + 1:] + ["--device", "cpu"])
    assert a.elastic_resume is True and a.resume == "auto" and a.checkpoint_every == 1


def test_residual_dtype_auto():
    """--residual-dtype auto: bf16 with --fp8 (the Megatron / TE fp8 recipe), fp32 otherwise."""
    import torch

    from nanodiloco_amd.trainer import _residual_dtype
    assert _residual_dtype("auto") == torch.float32
    assert _residual_dtype("auto", fp8=True) == torch.bfloat16
    assert _residual_dtype("fp32", fp8=True) == torch.float32
    assert _residual_dtype("bf16") == torch.bfloat16
    with pytest.raises(ValueError):
        _residual_dtype("fp16")


def test_trainer_runs_with_bf16_residual(tmp_path):
    """--residual-dtype bf16 through the trainer (CPU, synthetic data): DiLoCo inner + outer steps run and the
    model carries the bf16 residual stream."""
    import torch

    from nanodiloco_amd.trainer import TrainArgs, Trainer
    cfg = tmp_path / "m.json"
    cfg.write_text('{"hidden_size": 32, "intermediate_size": 64, "num_attention_heads": 2, '
                   '"num_hidden_layers": 1, "vocab_size": 32}')
    t = Trainer(TrainArgs(batch_size=4, per_device_batch_size=2, seq_length=16, warmup_steps=1, total_steps=4,
                          inner_steps=2, llama_config_file=str(cfg), wandb="off", device="cpu", data="synthetic",
                          residual_dtype="bf16"))
    assert t.model.residual_dtype == torch.bfloat16
    out = t.train()
    assert out["steps"] == 4 and out["outer_steps"] == 2
