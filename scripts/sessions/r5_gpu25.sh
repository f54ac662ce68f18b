#!/bin/bash
# round 5: bf16-only makespan plan -- interleaved 1B A/B (bf16 and fp8), plus the 150M default
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5y
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python bench.py --steps 8 --warmup 2 > $O/b150.log 2>&1 || { tail -5 $O/b150.log; exit 1; }
echo "150m $(tail -1 $O/b150.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
for rd in 1 2; do
  for a in "" "--fp8"; do
    for p in old cost; do
      ND_WGRAD_PLAN=$p timeout -k 10 400 python bench.py --model llama_1b.json --inner-steps 500 --steps 4 --warmup 2 $a > $O/b1${a}_${p}_$rd.log 2>&1 || { tail -5 $O/b1${a}_${p}_$rd.log; exit 1; }
      echo "1b $a plan=$p r$rd $(tail -1 $O/b1${a}_${p}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
