#!/bin/bash
# round 6 session 6: the down-dgrad + SwiGLU-backward GEMM touches its epilogue's gate / up lines during the K-loop
# (ND_DSW_GUPF, one LDS-DMA piece per wave in K-tiles nk-6 .. nk-3): GEMM GPU tests, then in-process A/B against
# the same source without it (gupf0) on the fused-epilogue GEMMs and on a Llama-150M fwd+bwd
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6f
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
A=nanodiloco_amd/_lib/alt
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo "== alt = gupf0 (speedup = alt/wt: >1 means the library WITHOUT the prefetch is SLOWER)"
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $A/libnd_kernels_gupf0.so --what epi --rounds 7 --iters 5 > $O/ab_epi.log 2>&1 || { tail -20 $O/ab_epi.log; exit 1; }
cat $O/ab_epi.log | grep -v amdgpu.ids
timeout -k 10 300 python -u scripts/ab_kernels.py --alt $A/libnd_kernels_gupf0.so --what step --rounds 5 --iters 3 > $O/ab_step.log 2>&1 || { tail -20 $O/ab_step.log; exit 1; }
grep fwd_bwd $O/ab_step.log
