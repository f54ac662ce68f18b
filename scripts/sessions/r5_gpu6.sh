#!/bin/bash
# round 5: kernel-trace of the bench step with and without the one-rank process group (where do the 2 % go?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5g
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
for arm in none rccl; do
  args=""; [ $arm = none ] && args="--backend none"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$arm -o run -- python3 bench.py --steps 3 --warmup 1 --wgrad-overlap 0 $args > $O/prof_$arm.log 2>&1 || { tail -5 $O/prof_$arm.log; exit 1; }
  f=$(find $O/prof_$arm -name "*kernel_stats.csv" | head -1); python3 scripts/prof_summary.py $f > $O/stats_$arm.md; head -14 $O/stats_$arm.md
  k=$(find $O/prof_$arm -name "*kernel_trace.csv" | head -1); cp $k $O/trace_$arm.csv
  tail -1 $O/prof_$arm.log | cut -c1-200
done
