"""Loader for the native HIP kernel library (``nanodiloco_amd/_lib/libnd_kernels.so``).

The library is a plain C ABI built by ``nanodiloco_amd/csrc/build.py`` with ``hipcc
--offload-arch=gfx950`` (no torch headers, no pybind, no hipify).  Kernels are launched on the
caller's current HIP stream, passed explicitly as a handle, so they interleave with PyTorch /
hipBLASLt work and are captured by hipGraphs like any other launch.

Policy: on a GPU tensor the HIP path is mandatory.  If the library is missing
we raise -- we never silently fall back to PyTorch on the GPU.  The PyTorch reference path is used
on CPU, or on GPU only when explicitly requested (``set_backend("torch")`` / ``--ops torch``).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(os.path.dirname(_HERE), "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libnd_kernels.so")
# profiling-only override: ND_KERNELS_LIB=<path> loads another build as THE library, e.g. the timing-ablation
# build (`python -m nanodiloco_amd.csrc.build --ablation` -> _lib/alt/libnd_kernels_ablation.so), whose
# wrong-result kernel variants the product library does not contain
LIB_PATH = os.environ.get("ND_KERNELS_LIB") or LIB_PATH

_lib = None
_lock = threading.Lock()
_backend = os.environ.get("NANODILOCO_OPS", "auto")  # auto | hip | torch


class ExtensionMissing(RuntimeError):
    pass


def set_backend(name: str):
    global _backend
    if name not in ("auto", "hip", "torch"):
        raise ValueError(name)
    _backend = name


def get_backend() -> str:
    return _backend


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ExtensionMissing(
                        f"HIP kernel library not found at {LIB_PATH}. Build it with "
                        f"`python -m nanodiloco_amd.csrc.build` (or __graft_entry__.build()).")
                raw = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
                _declare(raw)
                _lib = _StrictLib(raw)
    return _lib


def load_library(path: str) -> "_StrictLib":
    """Load another build of the kernel library side by side (RTLD_LOCAL) for in-process A/B."""
    raw = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    _declare(raw)
    return _StrictLib(raw)


class using:
    """``with _ext.using(other_lib): ...`` routes every op through `other_lib` (A/B benchmarking)."""

    def __init__(self, other):
        self.other = other

    def __enter__(self):
        global _lib
        self.prev = lib()
        _lib = self.other
        return self.other

    def __exit__(self, *exc):
        global _lib
        _lib = self.prev
        return False


def available() -> bool:
    try:
        lib()
        return True
    except (ExtensionMissing, OSError):
        return False


def use_hip(t: torch.Tensor) -> bool:
    """Decide the backend for an op whose primary input is ``t``."""
    if not t.is_cuda:
        if _backend == "hip":
            raise RuntimeError("backend 'hip' requested for a CPU tensor")
        return False
    if _backend == "torch":
        return False
    lib()  # raises loudly if missing: no silent eager fallback on the GPU
    return True


def stream_ptr(device: torch.device = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


DT_F32, DT_BF16 = 0, 1


def dtcode(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return DT_F32
    if t.dtype == torch.bfloat16:
        return DT_BF16
    raise TypeError(f"unsupported dtype {t.dtype}")


def _declare(L: ctypes.CDLL):
    """Argument types for every exported launcher (all return hipError_t as int)."""
    P, I, F, L64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64
    sigs = {
        "nd_version": [],
        # norms
        "nd_rmsnorm_fwd": [P, I, P, I, P, P, I, P, P, L64, I, F, P],
        "nd_rmsnorm_bwd": [P, I, P, I, P, P, P, P, I, P, L64, I, P, P],
        "nd_colsum_add": [P, P, I, I, P],
        "nd_rmsnorm_fwd_q": [P, I, P, I, P, P, I, P, P, L64, I, F, P, P, P, I, I, P],
        "nd_rmsnorm_bwd_q": [P, I, P, I, P, P, P, P, I, P, L64, I, P, P, P, P, I, I, P],
        "nd_transpose_bf16": [P, P, I, I, L64, L64, P],
        # rope (in place on packed qkv)
        "nd_rope_inplace": [P, I, P, P, L64, I, I, I, I, I, I, P],
        # attention
        "nd_attn_fwd": [P, P, P, P, P, I, I, I, I, I, L64, L64, P, P, F, P],
        "nd_attn_fwd_ks": [P, P, P, P, P, I, I, I, I, I, L64, L64, P, P, F, P, P],
        "nd_attn_bwd_ks": [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, L64, L64, P, P, F, I, P, P],
        "nd_attn_bwd_fused_ks": [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, L64, L64, P, P, F, I, P, P],
        "nd_attn_bwd_pre": [P, P, P, I, I, I, L64, L64, P],
        "nd_attn_bwd": [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, L64, L64, P, P, F, I, P],
        "nd_attn_bwd_fused": [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, L64, L64, P, P, F, I, P],
        # mlp
        "nd_swiglu_fwd": [P, P, I, L64, I, P],
        "nd_swiglu_bwd": [P, P, P, I, L64, I, P],
        "nd_swiglu_fwd_q": [P, P, L64, I, P, P, P, I, I, P],
        "nd_swiglu_bwd_q": [P, P, P, L64, I, P, P, P, I, I, P],
        # loss
        "nd_ce_fwd_bwd": [P, I, P, P, P, L64, I, I, P, P, F, P],
        "nd_ce_fwd_bwd_q8": [P, I, P, P, P, L64, I, I, P, P, P, P, P, I, I, P],
        # embedding
        "nd_embedding_fwd": [P, P, P, I, L64, I, I, P],
        "nd_embedding_bwd": [P, P, I, P, L64, I, I, P],
        "nd_embedding_bwd_sorted": [P, P, P, I, P, P, L64, I, I, P],
        # optimizer / outer step (flat buffers)
        "nd_sumsq_partial": [P, L64, P, I, P],
        "nd_adamw_step": [P, P, P, P, P, I, L64, P, I, F, F, F, F, F, F, F, F, P, I, P, P],
        "nd_pseudograd": [P, P, P, I, L64, P],
        "nd_outer_nesterov": [P, P, P, I, P, P, I, L64, F, F, F, I, P, P, P],
        "nd_axpby": [P, P, L64, F, F, P],
        # fp8 quantisation
        "nd_fp8_cast": [P, I, L64, P, P, I, P, I, P],
        "nd_fp8_cast_t": [P, I, I, I, L64, P, P, P, I, P, I, P],
        # projection GEMMs (C = A B^T) and their fused epilogues
        # ping-pong projection GEMMs (csrc/gemm_pp.hip)
        "nd_gemm_pp": [P, P, P, I, I, I, L64, L64, L64, P],
        "nd_gemm_pp_rope": [P, P, P, I, I, I, L64, L64, L64, P, P, I, I, I, P],
        "nd_gemm_pp_swiglu": [P, P, P, P, I, I, I, L64, L64, L64, L64, P],
        "nd_gemm_pp_dswiglu": [P, P, P, P, I, I, I, L64, L64, L64, L64, P],
        "nd_gemm_pp_f8": [P, P, P, I, I, I, L64, L64, L64, P, P, I, P],
        "nd_gemm_pp_rope_f8": [P, P, P, I, I, I, L64, L64, L64, P, P, P, P, I, I, I, P],
        "nd_gemm_pp_swiglu_f8": [P, P, P, P, I, I, I, L64, L64, L64, L64, P, P, P],
        "nd_gemm_pp_dswiglu_f8": [P, P, P, P, I, I, I, L64, L64, L64, L64, P, P, I, P],
        "nd_gemm_pp_set_group_m": [I],
        "nd_mlp_coef_set": [I],
        "nd_probe_tr8": [P, P, P, P],
        "nd_gemm_pp_swiglu_f8q": [P, P, P, P, I, I, I, L64, L64, L64, L64, P, P, P, P, I, P],
        "nd_gemm_pp_dswiglu_f8q": [P, P, P, P, I, I, I, L64, L64, L64, L64, P, P, I, P, P, I, P],
        "nd_wgrad_f8": [P, P, P, P, I, I, I, L64, L64, L64, P, P, I, P],
        "nd_gemm_pp_set_variant": [I],
        # one-wave-per-SIMD projection GEMM (csrc/gemm_w128.hip)
        "nd_gemm_w128": [P, P, P, I, I, I, L64, L64, L64, P],
        "nd_gemm_w128_set": [I, I, I],
        "nd_gemm_w128_set_ablation": [I],
        "nd_gemm_w128_set_vb": [I],
        # weight-gradient GEMM
        "nd_wgrad_splits": [I, I, I],
        "nd_wgrad_f8_splits": [I, I, I],
        "nd_wgrad_force_splits": [I],
        "nd_wgrad": [P, P, P, P, I, I, I, L64, L64, L64, P],
        "nd_wgrad2_splits": [I, I, I, I, I],
        "nd_wgrad2": [P, P, P, P, I, I, L64, L64, L64, P, P, P, P, I, I, L64, L64, L64, I, P],
    }
    for name, argtypes in sigs.items():
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int


class _StrictLib:
    """ctypes silently accepts surplus positional arguments (and then passes garbage through the
    C ABI); every launcher call is checked against its declared arity instead."""

    def __init__(self, raw):
        self._raw = raw
        self._fns = {}

    def __getattr__(self, name):
        f = self._fns.get(name)
        if f is None:
            fn = getattr(self._raw, name)
            n = len(fn.argtypes) if fn.argtypes is not None else None

            def f(*args, _fn=fn, _n=n, _name=name):
                if _n is not None and len(args) != _n:
                    raise TypeError(f"{_name}: expected {_n} arguments, got {len(args)}")
                return _fn(*args)

            self._fns[name] = f
        return f


def check(err: int, what: str):
    if err != 0:
        raise RuntimeError(f"{what} failed with hipError {err}")
