#!/bin/bash
# round 6 session 30: nt policy for the SwiGLU forward epilogue's direct (half-line) stores (ND_GEMM_PP_VARIANT=512):
# bitwise check + kernel A/B, then the bf16 step interleaved over 3 rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z4
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
VARIANTS=0,512 timeout -k 10 400 python -u scripts/store_policy_ab.py > $O/kernels.log 2>&1 || { tail -30 $O/kernels.log; exit 1; }
grep -E "bitwise|swiglu|total" $O/kernels.log
for r in 1 2 3; do
  for v in 0 512; do
    ND_GEMM_PP_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bf16_v${v}_r$r.log 2>&1 || { tail -20 $O/bf16_v${v}_r$r.log; exit 1; }
    echo "bf16 variant $v round $r: $(tail -1 $O/bf16_v${v}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
