#!/bin/bash
# round 6 session 25: the head_dim-64 dQ kernel at 3 waves / SIMD (168 VGPRs, no spill; the product build sits at 172
# VGPRs = 2 waves / SIMD): attention tests against the side build, in-process A/B of the raw attention and the step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6x
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
L=$(ls nanodiloco_amd/_lib/alt/libnd_kernels_*_dq3.so | head -1)
ND_KERNELS_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 200 --timeout-method thread > $O/attn_tests.log 2>&1 || { tail -30 $O/attn_tests.log; exit 1; }
echo "dq3 build: $(tail -1 $O/attn_tests.log)"
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $L --what attn --rounds 7 --iters 10 > $O/ab_attn.log 2>&1 || { tail -20 $O/ab_attn.log; exit 1; }
grep speedup $O/ab_attn.log
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $L --what attnk --rounds 7 --iters 10 > $O/ab_attnk.log 2>&1 || { tail -20 $O/ab_attnk.log; exit 1; }
grep speedup $O/ab_attnk.log
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $L --what step --rounds 5 --iters 3 > $O/ab_step.log 2>&1 || { tail -20 $O/ab_step.log; exit 1; }
grep speedup $O/ab_step.log
