#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "attention or hip_vs_torch or spike" > gpurun_out/attn_tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/attn_tests.log | cut -c1-160 | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/attn_thr_ab.py > gpurun_out/attn_ab.log 2>&1 || exit $?
cat gpurun_out/attn_ab.log
