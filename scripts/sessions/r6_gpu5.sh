#!/bin/bash
# round 6 session 5: serial kernel profiles of the bf16 and --fp8 bench steps at HEAD (after the attention wait
# fix), for the step breakdown and the fp8 cast share
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6e
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bf16 -o run -- python3 bench.py --steps 3 --warmup 1 --wgrad-overlap 0 > $O/prof_bf16.log 2>&1 || { tail -5 $O/prof_bf16.log; exit 1; }
f=$(find $O/prof_bf16 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats_bf16.md; head -24 $O/kernel_stats_bf16.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fp8 -o run -- python3 bench.py --fp8 --steps 3 --warmup 1 --wgrad-overlap 0 > $O/prof_fp8.log 2>&1 || { tail -5 $O/prof_fp8.log; exit 1; }
f=$(find $O/prof_fp8 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats_fp8.md; head -24 $O/kernel_stats_fp8.md
b() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rd in 1 2; do
  timeout -k 10 300 python bench.py > $O/bf16_$rd.log 2>&1 || { tail -5 $O/bf16_$rd.log; exit 1; }
  echo "bf16 r$rd $(b $O/bf16_$rd.log)"
  timeout -k 10 300 python bench.py --fp8 > $O/fp8_$rd.log 2>&1 || { tail -5 $O/fp8_$rd.log; exit 1; }
  echo "fp8 r$rd $(b $O/fp8_$rd.log)"
  timeout -k 10 300 python bench.py --residual-dtype bf16 > $O/bf16r_$rd.log 2>&1 || { tail -5 $O/bf16r_$rd.log; exit 1; }
  echo "bf16-residual r$rd $(b $O/bf16r_$rd.log)"
done
