#!/bin/bash
# round 3, session 50: micro-batch 128 vs 256 (bf16 and --fp8), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3aw
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  for mb in 128 256; do
    timeout -k 10 300 python bench.py --steps 6 --warmup 2 --micro-batch $mb > $O/bbf_${mb}_$r.log 2>&1 || exit 1
    echo "bf16 mb=$mb r=$r $(tail -1 $O/bbf_${mb}_$r.log | cut -c90-150)"
    timeout -k 10 300 python bench.py --steps 6 --warmup 2 --fp8 --micro-batch $mb > $O/bf8_${mb}_$r.log 2>&1 || exit 1
    echo "fp8 mb=$mb r=$r $(tail -1 $O/bf8_${mb}_$r.log | cut -c90-150)"
  done
done
