#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "wgrad" > gpurun_out/wgrad_tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/wgrad_tests.log | cut -c1-160 | tail -8
[ $rc -ne 0 ] && exit $rc
TOKENS=65536 VARIANTS=${VARIANTS:-dma0,4w,blas} timeout -k 10 400 python -u scripts/wgrad_bench.py > gpurun_out/wgrad_ab.log 2>&1 || exit $?
cat gpurun_out/wgrad_ab.log
