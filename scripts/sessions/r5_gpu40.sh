#!/bin/bash
# round 5: Llama-1B micro-batch 32 (auto) vs 64 sequences (fewer weight-gradient splits / slab passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5an
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rd in 1 2; do
  for mb in 32 64; do
    timeout -k 10 400 python bench.py --model llama_1b.json --inner-steps 500 --steps 4 --warmup 2 --micro-batch $mb > $O/b_${mb}_$rd.log 2>&1 || { tail -5 $O/b_${mb}_$rd.log; exit 1; }
    echo "mb=$mb r$rd $(tail -1 $O/b_${mb}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
