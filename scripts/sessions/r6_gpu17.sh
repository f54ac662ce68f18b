#!/bin/bash
# round 6 session 17: the one-wave-per-SIMD GEMM with its B operand staged through VGPRs (verdict r5 item 4,
# "make only one operand DMA-fed"): w128 GPU tests incl. the bitwise VB check, then the ten plain Llama-150M
# products at 131,072 tokens: hipBLASLt / pp / w128 / w128 (epilogue in last phase) / w128vb
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6p
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_w128_gpu.py -x -q --timeout 200 --timeout-method thread > $O/w128_tests.log 2>&1 || { tail -40 $O/w128_tests.log; exit 1; }
tail -1 $O/w128_tests.log
timeout -k 10 600 python -u scripts/gemm_pp_bench.py --tokens 131072 --rounds 3 > $O/gemm.log 2>&1 || { tail -30 $O/gemm.log; exit 1; }
grep -v "^round" $O/gemm.log | tail -14
