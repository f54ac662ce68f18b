#!/bin/bash
# round 3, session 16: ablations of the round-2 attention forward (what limits it)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3p
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
FWD_ONLY=1 VARIANTS=d,d:1,d:3,d:4,d:8,d:12,d:16,d:20,d:24,d:28,s1,r timeout -k 10 300 python -u scripts/attn_fwd_ab.py > $O/abl.log 2>&1; rc=$?; cat $O/abl.log; exit $rc
