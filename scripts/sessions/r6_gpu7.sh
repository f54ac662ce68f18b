#!/bin/bash
# round 6 session 7: fp8 cast kernel with 4 loads in flight per thread (A/B vs the committed HEAD library), then the
# serial kernel profiles of the bf16 and --fp8 bench steps and interleaved bench rounds (bf16 / --fp8 /
# --residual-dtype bf16) at the working tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6g
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
HEADLIB=$(ls nanodiloco_amd/_lib/alt/libnd_kernels_*_head.so | head -1)
echo "== alt = $HEADLIB (committed HEAD: no gate/up prefetch, one load per thread in the cast)"
timeout -k 10 200 python -u scripts/ab_kernels.py --alt $HEADLIB --what cast --rounds 7 --iters 10 > $O/ab_cast.log 2>&1 || { tail -20 $O/ab_cast.log; exit 1; }
grep cast_ $O/ab_cast.log
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/fp8_tests.log 2>&1 || { tail -30 $O/fp8_tests.log; exit 1; }
tail -2 $O/fp8_tests.log
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
