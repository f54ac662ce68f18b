#!/bin/bash
# round 5: longer Llama-150M loss-curve comparison, fp32 vs bf16 residual stream (2400 steps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bf
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u scripts/residual_convergence.py --steps 2400 --batch 32 --warmup 100 > $O/conv.log 2>&1 || { tail -20 $O/conv.log; exit 1; }
tail -3 $O/conv.log
