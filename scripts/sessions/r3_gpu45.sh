#!/bin/bash
# round 3, session 45: micro-batch 64 vs 128 at HEAD, bf16 (3 interleaved rounds) and --fp8 (1 more round)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3as
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2 3; do
  for mb in 64 128; do
    timeout -k 10 300 python bench.py --steps 8 --warmup 3 --micro-batch $mb > $O/bbf_${mb}_$r.log 2>&1 || exit 1
    echo "bf16 mb=$mb r=$r $(tail -1 $O/bbf_${mb}_$r.log | cut -c90-190)"
  done
done
for mb in 128 64; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 3 --fp8 --micro-batch $mb > $O/bf8_${mb}_3.log 2>&1 || exit 1
  echo "fp8 mb=$mb r=3 $(tail -1 $O/bf8_${mb}_3.log | cut -c90-190)"
done
