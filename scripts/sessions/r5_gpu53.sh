#!/bin/bash
# round 5: Llama-150M loss curves, fp32 vs bf16 residual stream, learnable synthetic data
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ba
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u scripts/residual_convergence.py --steps 600 --batch 32 > $O/conv.log 2>&1 || { tail -20 $O/conv.log; exit 1; }
tail -36 $O/conv.log
