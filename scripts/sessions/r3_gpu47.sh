#!/bin/bash
# round 3, session 47: lm-head logits chunk budget 4 GiB (2 chunks per 128-sequence micro-batch) vs 8 GiB (1 chunk)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3au
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  for mb in 4096 8192; do
    ND_CE_CHUNK_MB=$mb timeout -k 10 300 python bench.py --steps 8 --warmup 3 > $O/bbf_${mb}_$r.log 2>&1 || exit 1
    echo "bf16 ce=$mb r=$r $(tail -1 $O/bbf_${mb}_$r.log | cut -c90-190)"
    ND_CE_CHUNK_MB=$mb timeout -k 10 300 python bench.py --steps 8 --warmup 3 --fp8 > $O/bf8_${mb}_$r.log 2>&1 || exit 1
    echo "fp8 ce=$mb r=$r $(tail -1 $O/bf8_${mb}_$r.log | cut -c90-190)"
  done
done
