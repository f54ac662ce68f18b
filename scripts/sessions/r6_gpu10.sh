#!/bin/bash
# round 6 session 10: LDS-DMA pieces issued in bursts of four (m0 saved / restored once per burst, stepped by
# s_add) in the ping-pong projection and weight-gradient kernels: correctness tests, then in-process A/B against
# the same source built with -DND_DMA_BURST=0 (fused-epilogue GEMMs, weight gradients, fwd+bwd step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6j
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_gemm_pp_f8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pp_tests.log 2>&1 || { tail -40 $O/pp_tests.log; exit 1; }
tail -1 $O/pp_tests.log
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad" --timeout 200 --timeout-method thread > $O/wg_tests.log 2>&1 || { tail -40 $O/wg_tests.log; exit 1; }
tail -1 $O/wg_tests.log
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/fp8_tests.log 2>&1 || { tail -40 $O/fp8_tests.log; exit 1; }
tail -1 $O/fp8_tests.log
ALT=nanodiloco_amd/_lib/alt/libnd_kernels_burst0.so
echo "== alt = burst0 (speedup = alt/wt: >1 means the library WITHOUT the bursts is SLOWER)"
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $ALT --what epi --rounds 5 --iters 10 > $O/ab_epi.log 2>&1 || { tail -20 $O/ab_epi.log; exit 1; }
grep speedup $O/ab_epi.log
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $ALT --what wgrad --rounds 5 --iters 10 > $O/ab_wgrad.log 2>&1 || { tail -20 $O/ab_wgrad.log; exit 1; }
grep speedup $O/ab_wgrad.log
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $ALT --what step --rounds 5 --iters 3 > $O/ab_step.log 2>&1 || { tail -20 $O/ab_step.log; exit 1; }
grep speedup $O/ab_step.log
