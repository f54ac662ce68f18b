#!/bin/bash
# round 4, session 4: w128 DMA-issue variants (m0 handling, soffset form) against the kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4e}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/w128_probe.py ablate --abl ${ABL:-1,32,64} --rounds 5 > $O/ablate.log 2>&1
rc=$?; cat $O/ablate.log; exit $rc
