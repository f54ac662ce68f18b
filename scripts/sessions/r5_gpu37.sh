#!/bin/bash
# round 5: short-K plain products on the own kernel (--proj-gemm short: o fwd / dgrad, lm logits) -- removes the
# hipBLASLt fence before the o dgrad, so the grouped MLP weight gradient can co-run with the attention backward
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ak
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rd in 1 2 3; do
  for g in blas short; do
    timeout -k 10 200 python bench.py --steps 8 --warmup 2 --proj-gemm $g > $O/b_${g}_$rd.log 2>&1 || { tail -5 $O/b_${g}_$rd.log; exit 1; }
    echo "$g r$rd $(tail -1 $O/b_${g}_$rd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
