#!/bin/bash
# refresh the secondary README rows at round-2 HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2rows
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python bench.py --steps 5 --warmup 2 --model llama_1b.json --micro-batch 32 --fp8 --inner-steps 500 > gpurun_out/r2rows/b1b_fp8.log 2>&1 || exit $?
echo "1b fp8 $(tail -1 gpurun_out/r2rows/b1b_fp8.log | cut -c60-170)"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --model llama_default.json --micro-batch 8 --hip-graph > gpurun_out/r2rows/b10m.log 2>&1 || exit $?
echo "10m graph $(tail -1 gpurun_out/r2rows/b10m.log | cut -c60-200)"
