#!/bin/bash
# round 5: serial kernel profile of the --fp8 bench step at HEAD (bf16 residual by default)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bb
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --fp8 --steps 3 --warmup 1 --wgrad-overlap 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats.md; head -30 $O/kernel_stats.md
