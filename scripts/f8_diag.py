"""Diagnose the fp8 GEMM's element mapping: error pattern by output row / column residues."""
import torch
from nanodiloco_amd import ops
from nanodiloco_amd.ops import gemm as G
torch.manual_seed(0)
M = N = 256
K = 128
a = torch.randint(-2, 3, (M, K), device="cuda").float()
b = torch.randint(-2, 3, (N, K), device="cuda").float()
a8, b8 = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
one = torch.ones(1, device="cuda")
c = G.gemm_nt_f8(a8, b8, one, one).float()
e = a @ b.t()
bad = (c - e).abs() > 0.5
print("bad frac", bad.float().mean().item())
print("bad by row%32:", bad.float().view(8, 32, N).mean((0, 2)).tolist())
print("bad by col%32:", bad.float().view(M, 8, 32).mean((0, 1)).tolist())
print("bad by row//32:", bad.float().view(8, 32, N).mean((1, 2)).tolist())
print("bad by col//32:", bad.float().view(M, 8, 32).mean((0, 2)).tolist())
# which k-chunks: try a with only one nonzero k column
for kk in (0, 16, 31, 32, 48, 63, 64, 96, 127):
    a1 = torch.zeros(M, K, device="cuda"); a1[:, kk] = 1
    b1 = torch.zeros(N, K, device="cuda"); b1[:, kk] = 1
    c1 = G.gemm_nt_f8(a1.to(torch.float8_e4m3fn), b1.to(torch.float8_e4m3fn), one, one).float()
    print("k", kk, "sum", c1.sum().item(), "expect", M * N, "nonzero", (c1 != 0).sum().item())
r = (c - e)[:4, :40]
print(c[0, :40].tolist()); print(e[0, :40].tolist())
# which expected row does each output row hold (first 32-row block, first 32 columns)?
for r in range(32):
    d = (c[r:r + 1, :] - e[:64, :]).abs().sum(1)
    s = int(d.argmin())
    if s != r:
        print("row", r, "holds expected row", s, "(err %.1f)" % float(d[s]))
