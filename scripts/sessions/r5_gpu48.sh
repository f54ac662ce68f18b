#!/bin/bash
# round 5: PMC table of the Llama-1B bf16 step at HEAD (makespan split plan, auto micro-batch), plus its bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5av
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --model llama_1b.json --steps 3 --warmup 1 > $O/bench_1b.log 2>&1 || { tail -3 $O/bench_1b.log; exit 1; }
tail -1 $O/bench_1b.log | cut -c1-240
export ARGS="--model llama_1b.json --steps 1 --warmup 1"
bash scripts/sessions/r3_pmc.sh > $O/pmc1b.log 2>&1 || { tail -5 $O/pmc1b.log; exit 1; }
cp gpurun_out/pmc/merged.md $O/pmc_1b.md && head -22 $O/pmc_1b.md
