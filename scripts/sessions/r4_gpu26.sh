#!/bin/bash
# dK/dV prefetch depth A/B (64-query tiles, 2/3/4 LDS buffers) at the 150M and 1B GQA shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4ak
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -u scripts/attn_dkdv_nb.py > $O/nb_150m.log 2>&1; rc=$?; cat $O/nb_150m.log; [ $rc -eq 0 ] || exit $rc
B=16 NH=32 NKV=4 timeout -k 10 240 python -u scripts/attn_dkdv_nb.py > $O/nb_1b.log 2>&1; rc=$?; cat $O/nb_1b.log; exit $rc
