#!/bin/bash
# round 4, session 24: non-temporal gate / up loads in the down dgrad + SwiGLU-backward epilogue (pp variant
# 8192): kernel A/B, then in-step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4ah}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/gdma_ab.py --rounds 5 --pp-variant 8192 --wgrad-variant "" > $O/ab.log 2>&1
rc=$?; grep "dswiglu" $O/ab.log; [ $rc -eq 0 ] || { tail -5 $O/ab.log; exit $rc; }
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $O/d_$r.log 2>&1 || exit 1
  echo "default r=$r $(v $O/d_$r.log)"
  ND_GEMM_PP_VARIANT=8192 timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $O/n_$r.log 2>&1 || exit 1
  echo "nt gu loads r=$r $(v $O/n_$r.log)"
done
