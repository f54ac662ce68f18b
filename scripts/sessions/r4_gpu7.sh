#!/bin/bash
# round 4, session 7: weight-gradient kernel ablations (what its K-loop time is made of)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4o}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/wgrad_abl.py --abl ${ABL:-1,2,4,8,16,3,7,31} --rounds ${ROUNDS:-5} > $O/abl.log 2>&1
rc=$?; cat $O/abl.log; exit $rc
