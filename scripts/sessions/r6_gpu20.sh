#!/bin/bash
# round 6 session 20 (re-run as 20b with 8192 = no HBM stores): what the q|k|v + RoPE epilogue costs (ablation library: ND_GEMM_PP_VARIANT 8 = no epilogue,
# 16384 = RoPE math without the table loads) next to the plain ping-pong GEMM of the same product, and the MLP
# epilogues for reference
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export ND_KERNELS_LIB=nanodiloco_amd/_lib/alt/libnd_kernels_ablation.so
for v in 0 8 8192 0; do
  ND_GEMM_PP_VARIANT=$v timeout -k 10 200 python -u scripts/epi_abl.py > $O/epi_$v.log 2>&1 || { tail -20 $O/epi_$v.log; exit 1; }
  tail -1 $O/epi_$v.log
done
