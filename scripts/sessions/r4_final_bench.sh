#!/bin/bash
# round 4 closing validation, part 2: benches (bf16 x2, --fp8, Llama-1B bf16 / --fp8), kernel-trace profile of
# the bf16 bench, PMC table of the Llama-1B bf16 step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4final2}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
v() { python3 -c "
import json,sys
l=[x for x in open('$1') if x.startswith('{')][-1]; d=json.loads(l)
print(d['value'], d['ms_per_step'], d['model_tflops_per_gpu'], d['config']['micro_batch'], d['proj_gemm'], d.get('fp8_gemm'))"; }
for r in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$r.log 2>&1 || { tail -3 $O/bench_$r.log; exit 1; }
  echo "bf16 r=$r $(v $O/bench_$r.log)"
done
timeout -k 10 300 python bench.py --fp8 > $O/bench_fp8.log 2>&1 || exit 1
echo "fp8 $(v $O/bench_fp8.log)"
timeout -k 10 400 python bench.py --model llama_1b.json --steps 3 --warmup 1 > $O/bench_1b.log 2>&1 || exit 1
echo "1b bf16 $(v $O/bench_1b.log)"
timeout -k 10 400 python bench.py --model llama_1b.json --steps 3 --warmup 1 --fp8 > $O/bench_1b_fp8.log 2>&1 || exit 1
echo "1b fp8 $(v $O/bench_1b_fp8.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats.md; head -12 $O/kernel_stats.md
export ARGS="--model llama_1b.json --steps 1 --warmup 1"
bash scripts/sessions/r3_pmc.sh > $O/pmc1b.log 2>&1 || { tail -5 $O/pmc1b.log; exit 1; }
cp gpurun_out/pmc/merged.md $O/pmc_1b.md && head -20 $O/pmc_1b.md
