#!/bin/bash
# round 4, session 14: SPLIT LDS-DMA issue (half of each K-tile's pieces inside the MFMA phase) in the
# ping-pong kernels -- bitwise check + interleaved per-kernel A/B, then an in-step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${SESSION:-r4w}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/gdma_ab.py --rounds 5 --pp-variant 4096 --wgrad-variant a64 > $O/ab.log 2>&1
rc=$?; cat $O/ab.log; [ $rc -eq 0 ] || exit $rc
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $1 | tr '\n' ' '; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/base_$r.log 2>&1 || exit 1
  echo "default r=$r $(v $O/base_$r.log)"
  ND_GEMM_PP_VARIANT=4096 ND_WGRAD_VARIANT=a64 timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/split_$r.log 2>&1 || exit 1
  echo "split   r=$r $(v $O/split_$r.log)"
done
