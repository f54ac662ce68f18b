#!/bin/bash
# r2 session 5, call 1: GEMM kernel A/B vs hipBLASLt, full GPU tests, default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
set -o pipefail
timeout -k 10 300 python -u scripts/gemm_nt_bench.py --rounds 3 > gpurun_out/gemm_ab.log 2>&1 || exit $?
ND_GEMM_SCHED=0 timeout -k 10 300 python -u scripts/gemm_nt_bench.py --rounds 3 > gpurun_out/gemm_ab_s0.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
