#!/bin/bash
# round 4, session 12: fp8 defaults (auto dispatch + fp8 weight gradients) -- tests, interleaved bench A/B
# against bf16 and the own-kernel-only dispatch, and a kernel-trace profile of the fp8 default step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4t}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py tests/test_dispatch_cpu.py -x -q --timeout 300 --timeout-method thread > $O/fp8test.log 2>&1
rc=$?; tail -3 $O/fp8test.log; [ $rc -eq 0 ] || exit $rc
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/bf16_$r.log 2>&1 || { tail -3 $O/bf16_$r.log; exit 1; }
  echo "bf16 r=$r $(v $O/bf16_$r.log)"
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --fp8 > $O/f8auto_$r.log 2>&1 || { tail -3 $O/f8auto_$r.log; exit 1; }
  echo "fp8 auto r=$r $(v $O/f8auto_$r.log)"
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --fp8 --fp8-gemm pp > $O/f8pp_$r.log 2>&1 || { tail -3 $O/f8pp_$r.log; exit 1; }
  echo "fp8 pp-all r=$r $(v $O/f8pp_$r.log)"
done
timeout -k 10 400 python bench.py --model llama_1b.json --steps 3 --warmup 1 > $O/b1b.log 2>&1 || { tail -3 $O/b1b.log; exit 1; }
echo "1b bf16 $(v $O/b1b.log)"
timeout -k 10 400 python bench.py --model llama_1b.json --steps 3 --warmup 1 --fp8 > $O/b1b_f8.log 2>&1 || { tail -3 $O/b1b_f8.log; exit 1; }
echo "1b fp8 $(v $O/b1b_f8.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --fp8 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats.md; head -30 $O/kernel_stats.md
