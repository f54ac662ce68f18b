#!/bin/bash
# round 3, session 43: --fp8 step kernel profile (150M) and the Llama-1B --fp8 bench at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3aq
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python bench.py --steps 5 --warmup 2 --model llama_1b.json --micro-batch 32 --fp8 > $O/bench_1b_fp8.log 2>&1 && tail -1 $O/bench_1b_fp8.log | cut -c1-200 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --fp8 > $O/rocprof.log 2>&1; echo "rocprof rc $?"
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats.md; head -30 $O/kernel_stats.md
