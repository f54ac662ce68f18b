#!/bin/bash
# round 5 closing measurements at HEAD (after grouped wgrad + makespan plan): serial kernel profiles, PMC, Llama-1B H=500
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ai
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
for arm in bf16 fp8; do
  args="--wgrad-overlap 0"; [ $arm = fp8 ] && args="--fp8 --wgrad-overlap 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$arm -o run -- python3 bench.py --steps 3 --warmup 1 $args > $O/prof_$arm.log 2>&1 || { tail -5 $O/prof_$arm.log; exit 1; }
  f=$(find $O/prof_$arm -name "*kernel_stats.csv" | head -1); python3 scripts/prof_summary.py $f 30 > $O/stats_$arm.md
  head -8 $O/stats_$arm.md; grep -c Cijk $O/stats_$arm.md
done
bash scripts/sessions/r3_pmc.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
cp gpurun_out/pmc/merged.md $O/pmc_merged.md; head -22 $O/pmc_merged.md
for arm in bf16 fp8; do
  args=""; [ $arm = fp8 ] && args="--fp8"
  timeout -k 10 600 python bench.py --model llama_1b.json --inner-steps 500 --steps 3 --warmup 1 $args > $O/b1_$arm.log 2>&1 || { tail -3 $O/b1_$arm.log; exit 1; }
  tail -1 $O/b1_$arm.log | cut -c1-400
done
