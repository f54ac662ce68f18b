#!/bin/bash
# ping-pong GEMM start-stagger A/B (ND_GEMM_PP_STAGGER); attention forward packed-softmax variant (ND_ATTN_ABL=96)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4al
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/pp_stagger_ab.py --arms 1,2,4 > $O/stagger.log 2>&1; rc=$?; cat $O/stagger.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=d:32,d:96 FWD_ONLY=1 timeout -k 10 300 python -u scripts/attn_fwd_ab.py > $O/fwd96.log 2>&1; rc=$?; cat $O/fwd96.log; exit $rc
