#!/bin/bash
# round 3, session 30: after the unroll, the cheaper-mask / v_max3-tree variant (ABL 32) again
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ad
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
FWD_ONLY=1 VARIANTS=d,d:32,d,d:32 timeout -k 10 300 python -u scripts/attn_fwd_ab.py > $O/ab.log 2>&1; rc=$?; cat $O/ab.log; exit $rc
