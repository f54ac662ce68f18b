#!/bin/bash
# round 5: weight-gradient kernel time vs forced split count (isolated)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5at
mkdir -p $O
timeout -k 10 400 python scripts/wgrad_splits_ab.py > $O/ab.log 2>&1 || { tail -10 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
