#!/bin/bash
# round 5: Llama-1B with the new auto micro-batch (64) vs 32, bf16 and --fp8
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ao
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for a in "" "--fp8"; do
  for mb in auto 32; do
    timeout -k 10 400 python bench.py --model llama_1b.json --inner-steps 500 --steps 4 --warmup 2 --micro-batch $mb $a > $O/b${a}_${mb}.log 2>&1 || { tail -5 $O/b${a}_${mb}.log; exit 1; }
    echo "1b $a mb=$mb $(tail -1 $O/b${a}_${mb}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["micro_batch"])')"
  done
done
