#!/bin/bash
# round 5: fast sigmoid (v_rcp) in the SwiGLU epilogues -- in-process A/B against the previous library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5c
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
ALT=$(ls nanodiloco_amd/_lib/alt/libnd_kernels_7d55496.so)
timeout -k 10 300 python scripts/ab_kernels.py --alt $ALT --what epi --rounds 5 > $O/epi.log 2>&1 || { tail -5 $O/epi.log; exit 1; }
tail -12 $O/epi.log
timeout -k 10 300 python scripts/ab_kernels.py --alt $ALT --what step --rounds 4 --iters 3 > $O/step.log 2>&1 || { tail -5 $O/step.log; exit 1; }
tail -6 $O/step.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 > $O/rccl_$r.log 2>&1 || { tail -3 $O/rccl_$r.log; exit 1; }
  tail -1 $O/rccl_$r.log | cut -c1-140
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --backend none > $O/none_$r.log 2>&1 || { tail -3 $O/none_$r.log; exit 1; }
  tail -1 $O/none_$r.log | cut -c1-140
done
timeout -k 10 200 python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "swiglu or pp" > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; exit $rc
