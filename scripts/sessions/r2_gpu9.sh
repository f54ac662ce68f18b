#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|rror" gpurun_out/pytest_gpu.log | cut -c1-150 | tail -30
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
exit $rc
