#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u scripts/gemm_nt_bench.py --rounds 3 --only "qkv fwd,gu fwd,o fwd" --variants ${VARIANTS} > gpurun_out/gemm_abl.log 2>&1 || exit $?
cat gpurun_out/gemm_abl.log
