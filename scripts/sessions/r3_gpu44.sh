#!/bin/bash
# round 3, session 44: micro-batch A/B (Llama-1B 32 vs auto = 64; Llama-150M --fp8 64 vs 128), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ar
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  for mb in 32 auto; do
    timeout -k 10 400 python bench.py --steps 4 --warmup 2 --model llama_1b.json --micro-batch $mb > $O/b1b_${mb}_$r.log 2>&1 || exit 1
    echo "1b mb=$mb r=$r $(tail -1 $O/b1b_${mb}_$r.log | cut -c90-190)"
  done
  for mb in 64 128; do
    timeout -k 10 300 python bench.py --steps 8 --warmup 3 --fp8 --micro-batch $mb > $O/bf8_${mb}_$r.log 2>&1 || exit 1
    echo "fp8 mb=$mb r=$r $(tail -1 $O/bf8_${mb}_$r.log | cut -c90-190)"
  done
done
