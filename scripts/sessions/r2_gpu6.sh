#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "v6g4 or v5g0" > gpurun_out/gemm_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/gemm_nt_bench.py --rounds 3 --only "${ONLY:-qkv fwd,gu fwd,o fwd}" --variants ${VARIANTS} > gpurun_out/gemm_abl.log 2>&1 || exit $?
cat gpurun_out/gemm_abl.log
