#!/bin/bash
# round 5: where the fused-MLP epilogues spend their time (ablation library, timing only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5aa
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 0 8 4096 8192; do
  ND_KERNELS_LIB=$PWD/abl_r5.so ND_GEMM_PP_VARIANT=$v timeout -k 10 200 python scripts/epi_abl.py > $O/v$v.log 2>&1 || { tail -5 $O/v$v.log; exit 1; }
  cat $O/v$v.log
done
