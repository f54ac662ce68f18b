#!/bin/bash
# round 6 closing session (2/2): interleaved benches at HEAD (bf16, --fp8, --residual-dtype bf16; 20 timed steps)
# and Llama-1B H=500 (bf16, --fp8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
b() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rd in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bf16_$rd.log 2>&1 || { tail -5 $O/bf16_$rd.log; exit 1; }
  echo "bf16 r$rd $(b $O/bf16_$rd.log)"
  timeout -k 10 300 python bench.py --fp8 --steps 20 --warmup 3 > $O/fp8_$rd.log 2>&1 || { tail -5 $O/fp8_$rd.log; exit 1; }
  echo "fp8 r$rd $(b $O/fp8_$rd.log)"
  timeout -k 10 300 python bench.py --residual-dtype bf16 --steps 20 --warmup 3 > $O/bf16r_$rd.log 2>&1 || { tail -5 $O/bf16r_$rd.log; exit 1; }
  echo "bf16-residual r$rd $(b $O/bf16r_$rd.log)"
done
timeout -k 10 600 python bench.py --model llama_1b.json --inner-steps 500 --steps 3 --warmup 1 > $O/b1_bf16.log 2>&1 || { tail -3 $O/b1_bf16.log; exit 1; }
echo "1b bf16 $(b $O/b1_bf16.log)"
timeout -k 10 600 python bench.py --model llama_1b.json --inner-steps 500 --steps 3 --warmup 1 --fp8 > $O/b1_fp8.log 2>&1 || { tail -3 $O/b1_fp8.log; exit 1; }
echo "1b fp8 $(b $O/b1_fp8.log)"
