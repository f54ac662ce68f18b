#!/bin/bash
# round 5: does the 131k-token TunableOp table take effect on torch.mm?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ad
mkdir -p $O
timeout -k 10 300 python scripts/tuned_check.py nanodiloco_amd/tuning/_merged_probe.csv > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
cat $O/check.log | grep -v amdgpu.ids
