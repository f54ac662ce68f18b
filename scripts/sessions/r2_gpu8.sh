#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/gemm_tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/gemm_tests.log | cut -c1-120 | head -60
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/gemm_nt_bench.py --rounds 3 --variants ${VARIANTS:-1:0,5:4} > gpurun_out/gemm_ab4.log 2>&1 || exit $?
cat gpurun_out/gemm_ab4.log
