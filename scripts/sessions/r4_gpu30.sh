#!/bin/bash
# dQ kernel with 3 K / V LDS buffers (ND_ATTN_DQ_NB=3) vs the default 2, 150M and 1B GQA shapes; tests of the switch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4ao
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -u scripts/attn_dkdv_nb.py --env ND_ATTN_DQ_NB --arms 3 > $O/dq_150m.log 2>&1; rc=$?; cat $O/dq_150m.log; [ $rc -eq 0 ] || exit $rc
B=16 NH=32 NKV=4 timeout -k 10 240 python -u scripts/attn_dkdv_nb.py --env ND_ATTN_DQ_NB --arms 3 > $O/dq_1b.log 2>&1; rc=$?; cat $O/dq_1b.log; [ $rc -eq 0 ] || exit $rc
B=16 T=2048 timeout -k 10 240 python -u scripts/attn_dkdv_nb.py --env ND_ATTN_DQ_NB --arms 3 > $O/dq_2k.log 2>&1; rc=$?; cat $O/dq_2k.log; exit $rc
