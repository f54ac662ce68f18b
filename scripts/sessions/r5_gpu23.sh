#!/bin/bash
# round 5: makespan-model wgrad plan on the Llama-1B fp8 step (interleaved A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5w
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rd in 1 2; do
  for p in old cost; do
    ND_WGRAD_PLAN=$p timeout -k 10 400 python bench.py --model llama_1b.json --inner-steps 500 --steps 4 --warmup 2 --fp8 > $O/b1_${p}_$rd.log 2>&1 || { tail -5 $O/b1_${p}_$rd.log; exit 1; }
    echo "1b fp8 plan=$p r$rd $(tail -1 $O/b1_${p}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
