#!/bin/bash
# round 6 session 27: the q|k|v + RoPE epilogue with one position modulo per tile (T % 128 == 0) instead of one per row
# block and lane: RoPE GEMM tests, in-process A/B against the committed HEAD library (epilogue kernels, step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_gemm_pp_f8_gpu.py -x -q -k "rope" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
L=$(ls nanodiloco_amd/_lib/alt/libnd_kernels_*_head7.so | head -1)
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $L --what epi --rounds 7 --iters 5 > $O/ab_epi.log 2>&1 || { tail -20 $O/ab_epi.log; exit 1; }
grep speedup $O/ab_epi.log
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $L --what step --rounds 5 --iters 3 > $O/ab_step.log 2>&1 || { tail -20 $O/ab_step.log; exit 1; }
grep speedup $O/ab_step.log
