"""Llama causal LM over a flat :class:`ParamStore`.

Architecture and parameter names/shapes are exactly HF ``LlamaForCausalLM``
(HF/models/llama/modeling_llama.py:52-492), so checkpoints load into HF and HF
weights load here.  The compute graph is our own:

  h0  = embed(ids)                          fp32 residual stream, gathered from the fp32 master
  y   = rmsnorm(h0) * w_in[0]               compute dtype (bf16)
  per layer:
    qkv = rope(y @ [Wq|Wk|Wv]^T)            ONE GEMM (fused view of the flat buffer), RoPE in its epilogue
    o   = flash_attn(qkv)                   HIP kernel, reads packed qkv, writes [N, nh*hd]
    y,h = add_rmsnorm(h, o @ Wo^T, w_post)  residual add fused into the norm
    act = swiglu(y @ [Wgate|Wup]^T)         ONE GEMM, SwiGLU in its epilogue (SwiGLU backward in the
    y,h = add_rmsnorm(h, act @ Wdown^T, ..) down projection's dgrad epilogue)
  loss = lm_head_ce(y, W_lm, targets)       fused chunked GEMM + CE (+ its backward)

Weight gradients are written straight into ``store.grad`` by the ops' backward (and, for the
lm head, during the forward).  ``layer_hook(i)`` is called from the backward as soon as every
gradient in layer i's span is final (used for the inner-DDP bucketed all-reduce overlapped with
backward; see ``_GradHook`` for why the hook sits on the next norm's input).
"""
from __future__ import annotations

import dataclasses
from typing import Callable, List, Optional

import torch

from .. import ops
from ..config import LlamaConfig
from ..ops.cross_entropy import LM_KEY
from .param_store import ParamStore

_WARNED = set()


def _warn_once(key: str, msg: str) -> None:
    if key not in _WARNED:
        _WARNED.add(key)
        import warnings
        warnings.warn(msg, RuntimeWarning, stacklevel=3)


@dataclasses.dataclass
class CausalLMOutput:
    loss: Optional[torch.Tensor] = None
    logits: Optional[torch.Tensor] = None


class _GradHook(torch.autograd.Function):
    """Identity; calls ``fn(idx)`` when the gradient w.r.t. its input has been produced.

    Placement matters: autograd runs a node only after every consumer of its output has produced
    its gradient, so a hook on the INPUT of the add+RMSNorm that feeds layer i fires after the whole
    backward of layer i (GEMMs, attention, SwiGLU, both norms) -- i.e. when layer i's span of the
    flat grad buffer is final.  (A hook on a layer's OUTPUT would fire before that layer's own
    backward has run.)"""

    @staticmethod
    def forward(ctx, x, fn, idx):
        ctx.fn, ctx.idx = fn, idx
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        ops.join_wgrad()  # the layer's weight gradients may still be in flight on the side stream
        ctx.fn(ctx.idx)
        return g, None, None


class LlamaForCausalLM:
    def __init__(self, config: LlamaConfig, device="cpu", compute_dtype: torch.dtype = torch.float32,
                 store: Optional[ParamStore] = None, activation_checkpointing: bool = False, fp8: bool = False,
                 fp8_wgrad: bool = False, residual_dtype: Optional[torch.dtype] = None):
        self.config = config
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        # residual stream: fp32 (default, the autocast recipe) or bf16 (Megatron's default; ops/norm.py)
        self.residual_dtype = residual_dtype or torch.float32
        if self.residual_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("residual_dtype must be float32 or bfloat16")
        self.activation_checkpointing = activation_checkpointing
        L = config.num_hidden_layers
        groups = []
        for i in range(L):
            p = f"model.layers.{i}."
            groups.append([p + "self_attn.q_proj.weight", p + "self_attn.k_proj.weight", p + "self_attn.v_proj.weight"])
            groups.append([p + "mlp.gate_proj.weight", p + "mlp.up_proj.weight"])
        self.store = store or ParamStore(config.param_shapes(), device, compute_dtype, fuse_groups=groups)
        self._qkv_names = [g for g in groups[0::2]]
        self._gu_names = [g for g in groups[1::2]]
        self.layer_hook: Optional[Callable[[int], None]] = None
        # W^T copies for the input-gradient GEMMs (ops/linear.py), refreshed lazily whenever the
        # store's weight version moves: key -> [W^T buffer, version it holds, W view]
        self._wt_cache = {}
        self.training = True
        self.fp8 = None
        if fp8:
            if compute_dtype != torch.bfloat16 or self.device.type != "cuda":
                raise ValueError("fp8 needs bf16 compute on an MI355X")
            from ..ops.fp8 import Fp8Linears
            self.fp8 = Fp8Linears(self.device, wgrad_fp8=fp8_wgrad)

    # ------------------------------------------------------------------ init / io
    @torch.no_grad()
    def init_weights(self, seed: int = 1337):
        """HF ``_init_weights``: N(0, initializer_range) for Linear/Embedding, ones for RMSNorm."""
        std = self.config.initializer_range
        gen_dev = self.device if self.device.type == "cuda" else torch.device("cpu")
        g = torch.Generator(device=gen_dev)
        g.manual_seed(seed)
        for name in self.store.names:
            v = self.store.master_view(name)
            if v.dim() == 1:
                v.fill_(1.0)
            else:
                t = torch.empty(v.shape, dtype=torch.float32, device=gen_dev)
                t.normal_(0.0, std, generator=g)
                v.copy_(t)
        pad = self.config.pad_token_id
        if pad is not None:
            self.store.master_view("model.embed_tokens.weight")[pad].zero_()
        self.store.sync_shadow()
        return self

    def state_dict(self):
        return self.store.state_dict("master")

    def load_state_dict(self, sd, strict=True):
        self.store.load_state_dict(sd, strict=strict)

    def num_parameters(self) -> int:
        return self.store.num_params

    def train(self):
        self.training = True
        return self

    def eval(self):
        self.training = False
        return self

    def __call__(self, *a, **kw):
        return self.forward(*a, **kw)

    # ------------------------------------------------------------------ views
    def _w(self, name):  # compute-dtype weight (GEMM operand)
        return self.store.shadow_view(name)

    def _m(self, name):  # fp32 master weight (norms, embedding gather)
        return self.store.master_view(name)

    def _g(self, name):
        return self.store.grad_view(name) if self.training else None

    def _fused(self, names, which):
        if which == "grad" and not self.training:
            return None
        return self.store.fused_view(which, names)

    # ------------------------------------------------------------------ forward
    def _wt(self, key, w):
        """W^T (contiguous) for the dgrad GEMM, or None when the plain layout is used."""
        if not (self.training and w.is_cuda and w.dtype == torch.bfloat16 and ops.dgrad_transposed_enabled()):
            return None
        e = self._wt_cache.get(key)
        if e is None:
            e = [torch.empty(w.shape[1], w.shape[0], dtype=w.dtype, device=w.device), -1, w]
            self._wt_cache[key] = e
        if e[1] != self.store.version:
            ops.transpose_into(e[0], w)
            e[1] = self.store.version
        return e[0]

    def refresh_transposed(self):
        """Bring every cached W^T up to the current weights (eagerly, e.g. before a HIP-graph
        replay, whose captured GEMMs read these buffers but never re-run the version check)."""
        if not ops.dgrad_transposed_enabled():
            return
        for key, e in self._wt_cache.items():
            if e[1] != self.store.version:
                ops.transpose_into(e[0], e[2])
                e[1] = self.store.version

    def _fp8_on(self, key: str) -> bool:
        if self.fp8 is None:
            return False
        from ..ops.fp8 import fp8_projection
        return fp8_projection(key.split(".")[1])

    def _linear(self, key, x, w, gw, x8=None):
        if self._fp8_on(key):
            return self.fp8(key, x, w, gw, self.store.version, x8)
        return ops.linear(x, w, gw, self._wt(key, w))

    def _q8(self, key: str, grad: bool = False):
        """fp8 inner step: fused-producer quantisation target for projection ``key``'s input
        (``grad=False``) or output gradient (``grad=True``); None when not applicable."""
        if not self._fp8_on(key) or not self.training or not torch.is_grad_enabled():
            return None
        return self.fp8.dy_target(key) if grad else self.fp8.x_target(key)

    def _layer(self, i, h, y, cos, sin, B, T, next_norm, y8=None, kstart=None):
        c = self.config
        p = f"model.layers.{i}."
        cdt = self.compute_dtype
        eps = c.rms_norm_eps
        qn = self._qkv_names[i]
        w_qkv = self._fused(qn, "shadow")
        rope_cols = (c.num_attention_heads + c.num_key_value_heads) * c.head_dim
        fp8_qkv = self._fp8_on(f"{i}.qkv")
        wt_qkv = self._wt(f"{i}.qkv", w_qkv) if not fp8_qkv else None
        if not fp8_qkv and ops.linear_rope_supported(y, w_qkv, wt_qkv, c.head_dim, rope_cols):
            # own GEMM with RoPE on q|k in its epilogue: the attention skips its rotation pass
            qkv = ops.linear_rope(y, w_qkv, self._fused(qn, "grad"), wt_qkv, cos, sin, T, c.head_dim, rope_cols)
            rotated = True
        elif fp8_qkv and self.fp8.rope_ok(y, w_qkv, c.head_dim, rope_cols):
            # the same on the own fp8 GEMM (e4m3 operands, RoPE on the dequantised accumulator)
            qkv = self.fp8.rope(f"{i}.qkv", y, w_qkv, self._fused(qn, "grad"), self.store.version, y8, cos, sin, T,
                                c.head_dim, rope_cols)
            rotated = True
        else:
            if self.fp8 is not None and not fp8_qkv:
                _warn_once("qkv", "--fp8-keep-fused rope: the fused bf16 q|k|v + RoPE GEMM cannot run on this "
                                  "shape; the projection runs as a plain bf16 GEMM + separate RoPE pass (slower "
                                  "than fp8)")
            qkv = self._linear(f"{i}.qkv", y, w_qkv, self._fused(qn, "grad"), y8)
            rotated = False
        o = ops.attention(qkv, cos, sin, B, T, c.num_attention_heads, c.num_key_value_heads, c.head_dim,
                          inplace=True, kstart=kstart, rotated=rotated)
        a = self._linear(f"{i}.o", o, self._w(p + "self_attn.o_proj.weight"), self._g(p + "self_attn.o_proj.weight"))
        q_gu = self._q8(f"{i}.gu")
        y, h = ops.add_rmsnorm(h, a, self._m(p + "post_attention_layernorm.weight"),
                               self._g(p + "post_attention_layernorm.weight"), eps, cdt,
                               q8=q_gu, q8_bwd=self._q8(f"{i}.o", grad=True))
        gn = self._gu_names[i]
        w_gu = self._fused(gn, "shadow")
        w_dn = self._w(p + "mlp.down_proj.weight")
        if not self._fp8_on(f"{i}.gu"):
            wt_gu, wt_dn = self._wt(f"{i}.gu", w_gu), self._wt(f"{i}.down", w_dn)
            if ops.mlp_fused_supported(y, w_gu, wt_gu, w_dn, wt_dn):
                # own GEMMs with SwiGLU in the gate|up epilogue and its backward in the down dgrad's
                m = ops.mlp_fused(y, w_gu, self._fused(gn, "grad"), wt_gu, w_dn,
                                  self._g(p + "mlp.down_proj.weight"), wt_dn)
                return m, h
            if self.fp8 is not None:
                _warn_once("mlp", "--fp8-keep-fused mlp: the fused bf16 SwiGLU GEMMs cannot run on this shape; "
                                  "the MLP runs as plain bf16 GEMMs + separate SwiGLU passes (slower than fp8)")
        elif self.fp8.mlp_ok(y, w_gu, w_dn):
            # the same fusion on the own fp8 GEMMs
            m = self.fp8.mlp(f"{i}.gu", f"{i}.down", y, w_gu, w_dn, self._fused(gn, "grad"),
                             self._g(p + "mlp.down_proj.weight"), self.store.version,
                             q_gu.out if q_gu is not None else None)
            return m, h
        q_down = self._q8(f"{i}.down")
        gu = self._linear(f"{i}.gu", y, w_gu, self._fused(gn, "grad"), q_gu.out if q_gu is not None else None)
        act = ops.swiglu(gu, q8=q_down, q8_bwd=self._q8(f"{i}.gu", grad=True))
        m = self._linear(f"{i}.down", act, w_dn, self._g(p + "mlp.down_proj.weight"),
                         q_down.out if q_down is not None else None)
        return m, h

    def hidden_states(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Final-normed hidden states [B*T, d] in the compute dtype.  ``attention_mask`` (HF [B, T],
        left or right padded) becomes a per-sequence key start for the attention kernels."""
        c = self.config
        kstart = ops.key_start(attention_mask) if attention_mask is not None else None
        B, T = input_ids.shape
        cdt = self.compute_dtype
        eps = c.rms_norm_eps
        cos, sin = ops.rope_cache(T, c.head_dim, c.rope_theta, c.rope_scaling, self.device)
        h = ops.embedding(input_ids, self._m("model.embed_tokens.weight"), self._g("model.embed_tokens.weight"),
                          out_dtype=self.residual_dtype)
        hook = self.layer_hook if (self.layer_hook is not None and self.training and torch.is_grad_enabled()) else None
        if hook is not None:
            # layer 0's last gradient (its input_layernorm weight) is written by the backward of the
            # norm below; the hook node on the norm's INPUT runs right after that backward
            h = _GradHook.apply(h, hook, 0)
        q = self._q8("0.qkv")
        # (y, h): the embedding output feeds both the first norm and the residual stream; rmsnorm_res
        # fuses the two gradient contributions inside the norm's backward kernel
        y, h = ops.rmsnorm_res(h, self._m("model.layers.0.input_layernorm.weight"),
                               self._g("model.layers.0.input_layernorm.weight"), eps, cdt, q8=q)
        y8 = q.out if q is not None else None
        L = c.num_hidden_layers
        for i in range(L):
            nxt = f"model.layers.{i + 1}.input_layernorm.weight" if i + 1 < L else "model.norm.weight"
            if self.activation_checkpointing and self.training and torch.is_grad_enabled():
                from torch.utils.checkpoint import checkpoint
                m, h = checkpoint(self._layer, i, h, y, cos, sin, B, T, nxt, None, kstart, use_reentrant=False)
            else:
                m, h = self._layer(i, h, y, cos, sin, B, T, nxt, y8, kstart)
            if hook is not None and i + 1 < L:
                # layer i+1's gradients are final once the backward of the add+norm that produces its
                # input (and owns its input_layernorm weight) has run: hook that norm's input
                m = _GradHook.apply(m, hook, i + 1)
            q = self._q8(f"{i + 1}.qkv") if i + 1 < L else self._q8(LM_KEY)
            y, h = ops.add_rmsnorm(h, m, self._m(nxt), self._g(nxt), eps, cdt, q8=q,
                                   q8_bwd=self._q8(f"{i}.down", grad=True))
            y8 = q.out if q is not None else None
        # the final norm's fused e4m3 copy of y feeds the fp8 lm head (ops/cross_entropy.py); None otherwise
        self._lm_y8 = y8 if L > 0 else None
        return y

    def forward(self, input_ids: torch.Tensor, labels: Optional[torch.Tensor] = None, attention_mask=None,
                loss_scale: float = 1.0, return_logits: bool = False, targets: Optional[torch.Tensor] = None
                ) -> CausalLMOutput:
        """``labels`` follow HF semantics (shifted internally, -100 ignored).  ``attention_mask``
        follows HF too: pad keys are masked for every real token (left or right padding; pad positions
        should carry label -100, as the HF data path sets them)."""
        y = self.hidden_states(input_ids, attention_mask)
        lm = "lm_head.weight" if not self.config.tie_word_embeddings else "model.embed_tokens.weight"
        out = CausalLMOutput()
        if labels is not None or targets is not None:
            if targets is None:
                targets = ops.reference.shift_labels(labels, ops.IGNORE_INDEX)
            w_lm = self._w(lm)
            f8 = None
            if self._fp8_on(LM_KEY) and self.training and torch.is_grad_enabled():
                f8 = (self.fp8, self.store.version, getattr(self, "_lm_y8", None))
            out.loss = ops.lm_head_ce(y, w_lm, self._g(lm), targets.reshape(-1), loss_scale,
                                      wt=self._wt("lm_head", w_lm) if f8 is None else None, f8=f8)
            self._lm_y8 = None
        if return_logits or (labels is None and targets is None):
            with torch.no_grad():
                B, T = input_ids.shape
                out.logits = ops.mm_nt(y.detach(), self._w(lm)).float().view(B, T, -1)
        return out
