#!/bin/bash
# round 5: grouped MLP weight gradients on Llama-1B (interleaved A/B, 2 rounds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5u
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rd in 1 2; do
  for g in 0 1; do
    timeout -k 10 400 python bench.py --model llama_1b.json --inner-steps 500 --steps 4 --warmup 2 --wgrad-group $g > $O/b1_${g}_$rd.log 2>&1 || { tail -5 $O/b1_${g}_$rd.log; exit 1; }
    echo "1b group=$g r$rd $(tail -1 $O/b1_${g}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"])')"
  done
done
