#!/bin/bash
# weight-gradient GEMM: own wgrad_pp vs hipBLASLt addmm(out_dtype=float32) accumulate
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4am
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/wgrad_blas_ab.py > $O/wgrad_blas.log 2>&1; rc=$?; cat $O/wgrad_blas.log; exit $rc
