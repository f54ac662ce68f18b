#!/bin/bash
# round 4, session 20: weight-gradient side-stream overlap, 4 interleaved rounds (bf16), then Llama-1B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4ac}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $O/base_$r.log 2>&1 || exit 1
  echo "default r=$r $(v $O/base_$r.log)"
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --wgrad-overlap 1 > $O/wo_$r.log 2>&1 || exit 1
  echo "wgrad-overlap r=$r $(v $O/wo_$r.log)"
done
timeout -k 10 400 python bench.py --model llama_1b.json --steps 3 --warmup 1 > $O/b1b.log 2>&1 || exit 1
echo "1b default $(v $O/b1b.log)"
timeout -k 10 400 python bench.py --model llama_1b.json --steps 3 --warmup 1 --wgrad-overlap 1 > $O/b1b_wo.log 2>&1 || exit 1
echo "1b wgrad-overlap $(v $O/b1b_wo.log)"
