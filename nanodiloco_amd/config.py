"""Model / run configuration.

The JSON schema is the HF ``LlamaConfig`` kwargs schema that the reference feeds to
``LlamaConfig(**json)`` (REF/nanodiloco/main.py:97, REF/configs/llama_default.json:1-11);
fields the file omits take the HF defaults.  The run-metadata ("wandb")
config is a free-form dict (REF/configs/wandb_default.json:1-6).

We do not depend on ``transformers`` at runtime: :class:`LlamaConfig` is a plain dataclass that
accepts every HF key (unknown keys are kept in ``extra`` so a file round-trips unchanged).
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Any, Dict, Optional


def default_llama_config() -> Dict[str, Any]:
    """In-code default model (REF/nanodiloco/main.py:16-27): 6L / d128 / 4 heads / ff512."""
    return {
        "architectures": ["LlamaForCausalLM"],
        "hidden_size": 128,
        "intermediate_size": 512,
        "num_attention_heads": 4,
        "num_hidden_layers": 6,
        "rms_norm_eps": 1e-05,
        "use_cache": False,
    }


def default_run_config() -> Dict[str, Any]:
    """In-code default run-metadata config (REF/nanodiloco/main.py:29-35)."""
    return {"nodes": 1, "location": "local", "backend": "nccl", "measure_comms": True}


# Kept under the reference's name for API familiarity.
default_wandb_config = default_run_config


def load_config_from_file(path: str) -> Dict[str, Any]:
    """Plain JSON load (REF/nanodiloco/main.py:37-39)."""
    with open(path, "r") as f:
        return json.load(f)


_FIELDS_HF_DEFAULTS = dict(
    vocab_size=32000,
    hidden_size=4096,
    intermediate_size=11008,
    num_hidden_layers=32,
    num_attention_heads=32,
    num_key_value_heads=None,
    head_dim=None,
    hidden_act="silu",
    max_position_embeddings=2048,
    initializer_range=0.02,
    rms_norm_eps=1e-6,
    use_cache=True,
    pad_token_id=None,
    bos_token_id=1,
    eos_token_id=2,
    pretraining_tp=1,
    tie_word_embeddings=False,
    rope_theta=10000.0,
    rope_scaling=None,
    attention_bias=False,
    attention_dropout=0.0,
    mlp_bias=False,
)


@dataclasses.dataclass
class LlamaConfig:
    """HF-compatible Llama config (defaults = HF ``LlamaConfig``; HF/models/llama/configuration_llama.py)."""

    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: Optional[int] = None
    head_dim: Optional[int] = None
    hidden_act: str = "silu"
    max_position_embeddings: int = 2048
    initializer_range: float = 0.02
    rms_norm_eps: float = 1e-6
    use_cache: bool = True
    pad_token_id: Optional[int] = None
    bos_token_id: int = 1
    eos_token_id: int = 2
    pretraining_tp: int = 1
    tie_word_embeddings: bool = False
    rope_theta: float = 10000.0
    rope_scaling: Optional[Dict[str, Any]] = None
    attention_bias: bool = False
    attention_dropout: float = 0.0
    mlp_bias: bool = False
    architectures: Optional[list] = None
    extra: Dict[str, Any] = dataclasses.field(default_factory=dict)

    def __post_init__(self):
        if self.num_key_value_heads is None:
            self.num_key_value_heads = self.num_attention_heads
        if self.head_dim is None:
            self.head_dim = self.hidden_size // self.num_attention_heads
        # transformers>=5 stores rope_theta inside rope_parameters; accept both spellings.
        rp = self.extra.get("rope_parameters")
        if isinstance(rp, dict) and "rope_theta" in rp:
            self.rope_theta = float(rp["rope_theta"])
            if rp.get("rope_type", "default") != "default" and self.rope_scaling is None:
                self.rope_scaling = dict(rp)
        self.validate()

    # ------------------------------------------------------------------ helpers
    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "LlamaConfig":
        known = {f.name for f in dataclasses.fields(cls)} - {"extra"}
        kw = {k: v for k, v in d.items() if k in known}
        extra = {k: v for k, v in d.items() if k not in known}
        return cls(**kw, extra=extra)

    @classmethod
    def from_json(cls, path: str) -> "LlamaConfig":
        return cls.from_dict(load_config_from_file(path))

    def to_dict(self) -> Dict[str, Any]:
        d = dataclasses.asdict(self)
        extra = d.pop("extra")
        d.update(extra)
        d.pop("rope_parameters", None)
        if d.get("architectures") is None:
            d["architectures"] = ["LlamaForCausalLM"]
        return d

    def to_hf_json(self) -> Dict[str, Any]:
        """config.json content loadable by ``transformers.LlamaForCausalLM.from_pretrained``."""
        d = self.to_dict()
        d["model_type"] = "llama"
        d["torch_dtype"] = "float32"
        return d

    def validate(self):
        if self.hidden_act != "silu":
            raise ValueError(f"only hidden_act='silu' is supported, got {self.hidden_act}")
        if self.attention_bias or self.mlp_bias:
            raise ValueError("attention_bias / mlp_bias are not supported (reference uses none)")
        if self.num_attention_heads % self.num_key_value_heads:
            raise ValueError("num_attention_heads must be a multiple of num_key_value_heads")
        if self.rope_scaling not in (None, {}) and self.rope_scaling.get("rope_type", self.rope_scaling.get("type")) not in (
            "default", "linear", "llama3"):
            raise ValueError(f"unsupported rope_scaling {self.rope_scaling}")

    # ------------------------------------------------------------------ derived sizes
    @property
    def q_size(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_key_value_heads * self.head_dim

    def param_shapes(self):
        """Ordered (name, shape) list; order == HF ``state_dict`` order."""
        d, f, v = self.hidden_size, self.intermediate_size, self.vocab_size
        out = [("model.embed_tokens.weight", (v, d))]
        for i in range(self.num_hidden_layers):
            p = f"model.layers.{i}."
            out += [
                (p + "self_attn.q_proj.weight", (self.q_size, d)),
                (p + "self_attn.k_proj.weight", (self.kv_size, d)),
                (p + "self_attn.v_proj.weight", (self.kv_size, d)),
                (p + "self_attn.o_proj.weight", (d, self.q_size)),
                (p + "mlp.gate_proj.weight", (f, d)),
                (p + "mlp.up_proj.weight", (f, d)),
                (p + "mlp.down_proj.weight", (d, f)),
                (p + "input_layernorm.weight", (d,)),
                (p + "post_attention_layernorm.weight", (d,)),
            ]
        out.append(("model.norm.weight", (d,)))
        if not self.tie_word_embeddings:
            out.append(("lm_head.weight", (v, d)))
        return out

    def num_params(self) -> int:
        n = 0
        for _, s in self.param_shapes():
            k = 1
            for x in s:
                k *= x
            n += k
        return n

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs/token: 6·P_matmul + causal attention (fwd 2·2·T·d/2 per layer ×3 for bwd)."""
        d, L = self.hidden_size, self.num_hidden_layers
        p_mm = 0
        for name, s in self.param_shapes():
            if len(s) == 2 and "embed_tokens" not in name:
                p_mm += s[0] * s[1]
        attn = 12 * L * self.q_size * seq_len / 2  # causal: half the score matrix
        return 6.0 * p_mm + attn


def resolve_llama_config(path: Optional[str]) -> LlamaConfig:
    """Reference behaviour: JSON file if given else the in-code default (REF/nanodiloco/main.py:57)."""
    if path:
        if not os.path.exists(path):
            here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", path)
            if os.path.exists(here):
                path = here
        return LlamaConfig.from_json(path)
    return LlamaConfig.from_dict(default_llama_config())
