#!/bin/bash
# round 4, session 13: attention dK/dV ablations (what its time is made of)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4u}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/attn_dkdv_abl.py --rounds 5 > $O/abl.log 2>&1
rc=$?; cat $O/abl.log; exit $rc
