#!/bin/bash
# round 6 session 31: the plain products on the own ping-pong kernel in the step (--proj-gemm pp) against hipBLASLt
# (blas, default), interleaved over 3 rounds at the final HEAD (verdict r5 item 4's in-step criterion)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z5
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2 3; do
  for g in blas pp; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --proj-gemm $g > $O/bf16_${g}_r$r.log 2>&1 || { tail -20 $O/bf16_${g}_r$r.log; exit 1; }
    echo "proj-gemm $g round $r: $(tail -1 $O/bf16_${g}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["proj_gemm"])')"
  done
done
