#!/bin/bash
# round 6 session 14: wave-cycle segment stamps of the attention kernels incl. the dQ kernel (diagnostic build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6m
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u scripts/attn_stamps.py --lib nanodiloco_amd/_lib/alt/libnd_kernels_stamp.so > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
