#!/bin/bash
# GEMM variants: numerics (all epilogues x variants) then in-process timing A/B vs hipBLASLt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/gemm_nt_bench.py --rounds 3 --variants 1,3,4 > gpurun_out/gemm_ab2.log 2>&1 || exit $?
cat gpurun_out/gemm_ab2.log
