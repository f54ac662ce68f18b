#!/bin/bash
# round 6 session 16: the ping-pong weight-gradient epilogue made branch-free (buffer loads / stores) with the
# in-place C loads of a half issued up front: tests, then A/B against the committed HEAD library (incl. the
# one-split lm-head shape) and the step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6o
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py -x -q -k "wgrad" --timeout 200 --timeout-method thread > $O/wg_tests.log 2>&1 || { tail -40 $O/wg_tests.log; exit 1; }
tail -1 $O/wg_tests.log
HEADLIB=$(ls nanodiloco_amd/_lib/alt/libnd_kernels_*_head6.so | head -1)
echo "== alt = $HEADLIB (committed HEAD)"
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $HEADLIB --what wgrad --rounds 5 --iters 5 > $O/ab_wgrad.log 2>&1 || { tail -20 $O/ab_wgrad.log; exit 1; }
grep speedup $O/ab_wgrad.log
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $HEADLIB --what step --rounds 5 --iters 3 > $O/ab_step.log 2>&1 || { tail -20 $O/ab_step.log; exit 1; }
grep speedup $O/ab_step.log
