#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "attention or model or determin" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -5
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2prof/prof2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r2prof/rocprof2.log 2>&1 || exit $?
f=$(find gpurun_out/r2prof/prof2 -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 30 > gpurun_out/r2prof/kernel_stats2.md
grep attn gpurun_out/r2prof/kernel_stats2.md
