#!/bin/bash
# round 5: hipBLASLt workspace size (HIPBLASLT_WORKSPACE_SIZE, KiB) A/B on the bf16 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5bl
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
b() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rd in 1 2 3; do
  timeout -k 10 300 python bench.py > $O/d_$rd.log 2>&1 || { tail -5 $O/d_$rd.log; exit 1; }
  echo "default r$rd $(b $O/d_$rd.log)"
  HIPBLASLT_WORKSPACE_SIZE=262144 timeout -k 10 300 python bench.py > $O/w_$rd.log 2>&1 || { tail -5 $O/w_$rd.log; exit 1; }
  echo "ws256M r$rd $(b $O/w_$rd.log)"
done
