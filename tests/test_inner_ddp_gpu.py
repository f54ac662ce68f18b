"""Inner-DDP gradient sync on the MI355X: 2 ranks share one GPU over gloo (one GPU cannot host two
RCCL ranks), bf16 HIP kernels, the backward-overlapped per-layer all-reduce hooks (with and without
the side-stream weight-gradient GEMMs).  Same oracle as tests/test_inner_ddp_cpu.py: the synced
gradient equals the sum of every member's locally recomputed gradient.  (Tolerance, not bitwise:
the embedding backward accumulates with fp32 atomics, whose order varies run to run.)"""
import pytest
import torch

from ._mp import run_ranks
from .test_inner_ddp_cpu import _inner_sync

pytestmark = pytest.mark.gpu

GPU_CFG = dict(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_hidden_layers=3,
               vocab_size=1000, rms_norm_eps=1e-5)


@pytest.fixture(autouse=True)
def _gpu(hip_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run(rank, world, wgrad_overlap):
    from nanodiloco_amd import ops
    ops.set_wgrad_overlap(wgrad_overlap)
    return _inner_sync(rank, world, 2, True, GPU_CFG, True, 1e-4, 128)


@pytest.mark.parametrize("wgrad_overlap", [0, 1])
def test_inner_ddp_hooks_on_gpu(wgrad_overlap):
    assert all(run_ranks(_run, 2, wgrad_overlap, timeout=120))
