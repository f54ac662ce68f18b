#!/bin/bash
# round 3, session 35: fused-epilogue configurations at HEAD, interleaved bench A/B (2 rounds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ai
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  for cfg in "1 1" "0 1" "1 0" "0 0"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --fused-rope $1 --fused-mlp $2 > $O/bench_$1$2_$r.log 2>&1 || exit 1
    echo "rope=$1 mlp=$2 round $r: $(tail -1 $O/bench_$1$2_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
