#!/bin/bash
# round 5: own ping-pong GEMM vs hipBLASLt as a function of the token count (L2 / MALL-resident vs HBM-streamed A)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5s
mkdir -p $O
for t in 8192 32768 131072; do
  timeout -k 10 300 python scripts/gemm_pp_bench.py --tokens $t --rounds 3 > $O/tok_$t.log 2>&1 || { tail -5 $O/tok_$t.log; exit 1; }
  echo "== tokens $t"; grep -E "^(qkv|o |gu|down|lm|total)" $O/tok_$t.log | sed -e 's/| w128o.*//' 
done
