#!/bin/bash
# round 6 session 8: the dK/dV kernel writes the e5m2 d(q|k|v) of the fp8 step (dK / dV from its stores, dQ
# re-read): bitwise tests, attention tests, the --fp8 kernel profile, interleaved --fp8 bench A/B (ND_ATTN_Q8=0/1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6h
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/fp8_tests.log 2>&1 || { tail -40 $O/fp8_tests.log; exit 1; }
tail -2 $O/fp8_tests.log
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 200 --timeout-method thread > $O/attn_tests.log 2>&1 || { tail -40 $O/attn_tests.log; exit 1; }
tail -2 $O/attn_tests.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fp8 -o run -- python3 bench.py --fp8 --steps 3 --warmup 1 --wgrad-overlap 0 > $O/prof_fp8.log 2>&1 || { tail -5 $O/prof_fp8.log; exit 1; }
f=$(find $O/prof_fp8 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py $f > $O/kernel_stats_fp8.md; head -30 $O/kernel_stats_fp8.md
b() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rd in 1 2 3; do
  ND_ATTN_Q8=1 timeout -k 10 300 python bench.py --fp8 > $O/q8on_$rd.log 2>&1 || { tail -5 $O/q8on_$rd.log; exit 1; }
  echo "fp8 attn-q8 on  r$rd $(b $O/q8on_$rd.log)"
  ND_ATTN_Q8=0 timeout -k 10 300 python bench.py --fp8 > $O/q8off_$rd.log 2>&1 || { tail -5 $O/q8off_$rd.log; exit 1; }
  echo "fp8 attn-q8 off r$rd $(b $O/q8off_$rd.log)"
done
