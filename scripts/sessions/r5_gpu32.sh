#!/bin/bash
# round 5: which kernels run under the 131k TunableOp table (kernel stats of tuned_check.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5af
mkdir -p $O
export TMPDIR=/tmp
cp gpurun_out/r5ae/merged.csv $O/merged.csv 2>/dev/null || cp nanodiloco_amd/tuning/_merged_probe.csv $O/merged.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/tuned_check.py $O/merged.csv > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 scripts/prof_summary.py $f 12
