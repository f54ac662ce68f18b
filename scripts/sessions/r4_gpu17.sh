#!/bin/bash
# round 4, session 17: software-pipelined dK/dV (one wave per SIMD) vs the default kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4z}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/attn_dkdv_sp_ab.py --rounds 5 > $O/ab.log 2>&1
rc=$?; cat $O/ab.log; exit $rc
