#!/bin/bash
# round 4, session 1: one-wave-per-SIMD GEMM (csrc/gemm_w128.hip) -- numerics, then per-shape A/B
# against hipBLASLt and the ping-pong kernel at 131,072 tokens
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4a}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_w128_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -5 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/gemm_pp_bench.py --tokens 131072 --rounds 3 > $O/bench.log 2>&1
rc=$?; tail -16 $O/bench.log; exit $rc
