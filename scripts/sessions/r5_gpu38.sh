#!/bin/bash
# round 5: makespan-plan threshold 99 % (q|k|v weight gradient 16 splits = 3 full waves instead of 5 = 240 workgroups)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5al
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rd in 1 2 3; do
  for p in c90 c99; do
    ND_WGRAD_PLAN=$p timeout -k 10 200 python bench.py --steps 8 --warmup 2 > $O/b_${p}_$rd.log 2>&1 || { tail -5 $O/b_${p}_$rd.log; exit 1; }
    echo "$p r$rd $(tail -1 $O/b_${p}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
