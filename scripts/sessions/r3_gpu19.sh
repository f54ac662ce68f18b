#!/bin/bash
# round 3, session 19: phase timing of the ping-pong attention forward
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u scripts/attn_diag.py > $O/diag.log 2>&1; rc=$?; cat $O/diag.log; exit $rc
