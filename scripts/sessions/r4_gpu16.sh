#!/bin/bash
# round 4, session 16: bf16 step A/B -- plain projection / lm-head GEMMs on hipBLASLt (default) vs the own
# ping-pong (pp) and one-wave-per-SIMD (w128) kernels, and a HIP-graph captured micro-step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4y}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2; do
  for arm in blas pp w128 graph; do
    if [ $arm = graph ]; then extra="--hip-graph"; else extra="--proj-gemm $arm"; fi
    timeout -k 10 300 python bench.py --steps 6 --warmup 2 $extra > $O/${arm}_$r.log 2>&1 || { tail -3 $O/${arm}_$r.log; exit 1; }
    echo "$arm r=$r $(v $O/${arm}_$r.log)"
  done
done
