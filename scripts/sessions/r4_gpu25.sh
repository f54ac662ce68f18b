#!/bin/bash
# round 4, session 25: micro-batch A/B for the fp8 step (128 = auto vs 256 vs 64)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4ai}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2; do
  for mb in 128 256 64; do
    timeout -k 10 300 python bench.py --steps 6 --warmup 2 --fp8 --micro-batch $mb > $O/f8_${mb}_$r.log 2>&1 || exit 1
    echo "fp8 mb=$mb r=$r $(v $O/f8_${mb}_$r.log)"
  done
done
