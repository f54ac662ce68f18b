"""Pins the gfx950 `ds_read_b64_tr_b8` semantics the fp8 weight-gradient kernel relies on (the ISA text
is not available in this image): per 16-lane group, lane 2q + p supplies the address of 8 bytes of row q
(q = 0..7) at columns 8p .. 8p + 7 of a [8 rows][16 columns] byte block, and lane i of the group receives
column i of the 8 rows, row q in byte q."""
import pytest
import torch

from nanodiloco_amd.ops import _ext

pytestmark = pytest.mark.gpu


def _tr8(data: torch.Tensor, addr: torch.Tensor) -> torch.Tensor:
    out = torch.zeros(128, dtype=torch.int32, device="cuda")
    _ext.check(_ext.lib().nd_probe_tr8(_ext.ptr(data), _ext.ptr(addr), _ext.ptr(out),
                                       _ext.stream_ptr(data.device)), "nd_probe_tr8")
    return out.view(torch.uint8).view(64, 8).cpu()


def _src_index(addr: torch.Tensor) -> torch.Tensor:
    """[64 lanes][8 bytes] -> LDS byte index each output byte came from (two runs: low / high byte)."""
    idx = torch.arange(4096, device="cuda")
    lo = _tr8((idx & 255).to(torch.uint8), addr).long()
    hi = _tr8((idx >> 8).to(torch.uint8), addr).long()
    return hi * 256 + lo


def test_tr8_block_transpose(hip_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ld = 128  # LDS row pitch (bytes) of a [32 rows][128 B] image (the probe holds 4 KiB)
    lane = torch.arange(64)
    g, j = lane // 16, lane % 16
    q, p = j // 2, j % 2
    # group g reads the block at rows 8 g .. 8 g + 7, columns 0 .. 15
    addr = ((8 * g + q) * ld + 8 * p).int().cuda()
    src = _src_index(addr)
    exp = torch.empty(64, 8, dtype=torch.long)
    for l in range(64):
        for b in range(8):
            exp[l, b] = (8 * (l // 16) + b) * ld + (l % 16)
    if not torch.equal(src, exp):
        print("tr8 source indices, lanes 0-17:", src[:18].tolist())
    assert torch.equal(src, exp)
