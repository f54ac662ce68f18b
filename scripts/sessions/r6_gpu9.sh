#!/bin/bash
# round 6 session 9: the Q8 dK/dV epilogue with the dQ loads issued first and one amax atomic per workgroup:
# isolated A/B (bwd + separate cast vs bwd writing e5m2), bitwise fp8 tests, interleaved --fp8 bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6i
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u scripts/attn_q8_bench.py > $O/q8_iso.log 2>&1 || { tail -20 $O/q8_iso.log; exit 1; }
cat $O/q8_iso.log
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py -x -q -k "q8 or fused" --timeout 200 --timeout-method thread > $O/fp8_tests.log 2>&1 || { tail -40 $O/fp8_tests.log; exit 1; }
tail -2 $O/fp8_tests.log
b() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rd in 1 2 3; do
  ND_ATTN_Q8=1 timeout -k 10 300 python bench.py --fp8 > $O/q8on_$rd.log 2>&1 || { tail -5 $O/q8on_$rd.log; exit 1; }
  echo "fp8 attn-q8 on  r$rd $(b $O/q8on_$rd.log)"
  ND_ATTN_Q8=0 timeout -k 10 300 python bench.py --fp8 > $O/q8off_$rd.log 2>&1 || { tail -5 $O/q8off_$rd.log; exit 1; }
  echo "fp8 attn-q8 off r$rd $(b $O/q8off_$rd.log)"
done
