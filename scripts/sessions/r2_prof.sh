#!/bin/bash
# Round-2 measurement session: default bench, fp8, 1B, then a rocprofv3 kernel profile of the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
set -o pipefail
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r2prof/bench_bf16.log 2>&1 || exit $?
tail -1 gpurun_out/r2prof/bench_bf16.log | cut -c1-160
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --fp8 > gpurun_out/r2prof/bench_fp8.log 2>&1 || exit $?
tail -1 gpurun_out/r2prof/bench_fp8.log | cut -c1-160
timeout -k 10 500 python bench.py --steps 5 --warmup 2 --model llama_1b.json --micro-batch 32 > gpurun_out/r2prof/bench_1b.log 2>&1 || exit $?
tail -1 gpurun_out/r2prof/bench_1b.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2prof/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r2prof/rocprof.log 2>&1 || exit $?
f=$(find gpurun_out/r2prof/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 30 > gpurun_out/r2prof/kernel_stats.md
head -20 gpurun_out/r2prof/kernel_stats.md
