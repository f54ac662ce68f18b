#!/bin/bash
# Round-2 final validation at HEAD: full GPU test suite, smoke(), benches, kernel profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/final/pytest_gpu.log | cut -c1-200 | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/final/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/final/bench_default.log | cut -c1-200
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --fp8 > gpurun_out/final/bench_fp8.log 2>&1 || exit $?
tail -1 gpurun_out/final/bench_fp8.log | cut -c1-200
timeout -k 10 500 python bench.py --steps 5 --warmup 2 --model llama_1b.json --micro-batch 32 > gpurun_out/final/bench_1b.log 2>&1 || exit $?
tail -1 gpurun_out/final/bench_1b.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/final/rocprof.log 2>&1 || exit $?
f=$(find gpurun_out/final/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" 30 > gpurun_out/final/kernel_stats.md
head -16 gpurun_out/final/kernel_stats.md
