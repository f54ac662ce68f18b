#!/bin/bash
# round 5: grouped MLP weight gradients, serial (--wgrad-overlap 0) interleaved A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5r
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rd in 1 2 3; do
  for g in 0 1; do
    timeout -k 10 200 python bench.py --steps 8 --warmup 2 --wgrad-group $g --wgrad-overlap 0 > $O/b_${g}_$rd.log 2>&1 || { tail -5 $O/b_${g}_$rd.log; exit 1; }
    echo "serial group=$g round=$rd $(tail -1 $O/b_${g}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
