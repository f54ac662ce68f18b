#!/bin/bash
# kernel-trace profile of the bf16 bench step with the weight-gradient side stream off (--wgrad-overlap 0): with it on,
# concurrent kernels' trace durations overlap and do not add up to the step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4final2}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof0 -o run -- python3 bench.py --steps 3 --warmup 1 --wgrad-overlap 0 > $O/prof0.log 2>&1 || { tail -5 $O/prof0.log; exit 1; }
f=$(find $O/prof0 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats_serial.md; head -30 $O/kernel_stats_serial.md
