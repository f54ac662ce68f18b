#!/bin/bash
# round 6 session 26: Llama-1B (H = 500) bf16 and --fp8 at HEAD (SwiGLU coefficient form), as the round-6 closing runs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6y
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench.py --model llama_1b.json --inner-steps 500 --steps 3 --warmup 1 > $O/b1_bf16.log 2>&1 || { tail -3 $O/b1_bf16.log; exit 1; }
tail -1 $O/b1_bf16.log | cut -c1-200
timeout -k 10 600 python bench.py --model llama_1b.json --inner-steps 500 --steps 3 --warmup 1 --fp8 > $O/b1_fp8.log 2>&1 || { tail -3 $O/b1_fp8.log; exit 1; }
tail -1 $O/b1_fp8.log | cut -c1-200
