"""Hot-path ops.  Each op dispatches to a hand-written HIP/CDNA4 kernel for GPU tensors and to the
PyTorch reference (``ops.reference``) for CPU tensors; see ``ops/_ext.py`` for the policy."""
from ._ext import available as hip_available, set_backend, get_backend, ExtensionMissing
from .linear import linear, wgrad_accumulate, set_wgrad_overlap, wgrad_overlap_enabled, join_wgrad, \
    set_dgrad_transposed, dgrad_transposed_enabled, transpose_into, mm_nt, set_proj_gemm, proj_gemm, \
    set_fused_epilogues, fused_epilogues, linear_rope, linear_rope_supported, mlp_fused, mlp_fused_supported, \
    set_wgrad_group, wgrad_group_enabled
from .norm import rmsnorm, rmsnorm_res, add_rmsnorm
from .embedding import embedding
from .swiglu import swiglu
from .attention import attention, rope_cache, set_attn_fused_stats, key_start, check_padding
from .cross_entropy import lm_head_ce, IGNORE_INDEX
from .optim import adamw_step, global_grad_norm, pseudograd, outer_nesterov
from .determinism import set_deterministic, deterministic
from . import reference

__all__ = ["hip_available", "set_backend", "get_backend", "ExtensionMissing", "linear", "wgrad_accumulate",
           "set_wgrad_overlap", "wgrad_overlap_enabled", "join_wgrad", "set_wgrad_group", "wgrad_group_enabled",
           "set_dgrad_transposed", "dgrad_transposed_enabled", "transpose_into",
           "rmsnorm", "rmsnorm_res", "add_rmsnorm", "set_attn_fused_stats", "embedding", "swiglu", "attention", "rope_cache", "lm_head_ce",
           "IGNORE_INDEX", "adamw_step", "global_grad_norm", "pseudograd", "outer_nesterov", "reference"]
