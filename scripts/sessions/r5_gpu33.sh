#!/bin/bash
# round 5: cost of the bitwise-deterministic step (--deterministic: sorted embedding backward, per-row loss sum)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ag
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rd in 1 2 3; do
  for d in 0 1; do
    extra=""; [ $d = 1 ] && extra="--deterministic"
    timeout -k 10 200 python bench.py --steps 8 --warmup 2 $extra > $O/b_${d}_$rd.log 2>&1 || { tail -5 $O/b_${d}_$rd.log; exit 1; }
    echo "det=$d r$rd $(tail -1 $O/b_${d}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["deterministic"])')"
  done
done
