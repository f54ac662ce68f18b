#!/bin/bash
# round 4, session 19: step-level knobs A/B (bf16): weight-gradient GEMMs on a side stream, ping-pong tile
# group size
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4ab}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/base_$r.log 2>&1 || exit 1
  echo "default r=$r $(v $O/base_$r.log)"
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --wgrad-overlap 1 > $O/wo_$r.log 2>&1 || exit 1
  echo "wgrad-overlap r=$r $(v $O/wo_$r.log)"
  ND_GEMM_PP_GM=8 timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/gm8_$r.log 2>&1 || exit 1
  echo "pp GM=8 r=$r $(v $O/gm8_$r.log)"
  ND_GEMM_PP_GM=2 timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/gm2_$r.log 2>&1 || exit 1
  echo "pp GM=2 r=$r $(v $O/gm2_$r.log)"
done
