#!/bin/bash
# round 6 session 1: own-RCCL failure paths (non-blocking init timeout, abort, bounded destroy) + the
# attention softmax-arithmetic experiments (ND_ATTN_X side libraries: 1 setprio S chains, 2 packed f32,
# 4 polynomial exp2 for 1/8 of the forward's exps, 8 setprio second chains, 9 = 1|8, 3 = 1|2, slp = SLP on)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6a
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_rccl_gpu.py -s > $O/rccl.log 2>&1 || { tail -40 $O/rccl.log; exit 1; }
tail -25 $O/rccl.log
for v in x1 x2 x3 x4 x8 x9 slp; do
  echo "== alt = ND_ATTN_X $v (speedup = alt/wt: >1 means the variant is SLOWER than the product build)"
  timeout -k 10 180 python -u scripts/ab_kernels.py --alt nanodiloco_amd/_lib/alt/libnd_kernels_$v.so --what attnk --rounds 5 --iters 10 > $O/ab_$v.log 2>&1 || { tail -20 $O/ab_$v.log; exit 1; }
  cat $O/ab_$v.log
done
