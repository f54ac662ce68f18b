#!/bin/bash
# round 3, session 48: TunableOp search for the 128-sequence micro-batch GEMM shapes of Llama-150M
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3av
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=$O/tuned_128.csv MAX_MS=40 timeout -k 10 600 python -u scripts/tune_gemms.py llama_150m.json:128 > $O/tune.log 2>&1; rc=$?; tail -3 $O/tune.log; exit $rc
