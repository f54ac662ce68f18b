#!/bin/bash
# Llama-1B micro-batch 32 (auto) vs 64, interleaved, bf16
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4aq
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { python3 -c "
import json
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step'], d['config']['micro_batch'])"; }
for r in 1 2; do
  timeout -k 10 400 python bench.py --model llama_1b.json --steps 3 --warmup 1 > $O/mb32_$r.log 2>&1 || { tail -3 $O/mb32_$r.log; exit 1; }
  echo "auto r=$r $(v $O/mb32_$r.log)"
  timeout -k 10 400 python bench.py --model llama_1b.json --steps 3 --warmup 1 --micro-batch 64 > $O/mb64_$r.log 2>&1 || { tail -3 $O/mb64_$r.log; exit 1; }
  echo "64   r=$r $(v $O/mb64_$r.log)"
done
