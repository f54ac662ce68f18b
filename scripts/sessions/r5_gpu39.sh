#!/bin/bash
# round 5: serial kernel profile of the Llama-1B bf16 step (H=500, micro-batch 32)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5am
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --model llama_1b.json --inner-steps 500 --steps 2 --warmup 1 --wgrad-overlap 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 scripts/prof_summary.py $f 30 > $O/stats.md
cat $O/stats.md
