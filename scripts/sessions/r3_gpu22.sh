#!/bin/bash
# round 3, session 22: DSWIGLU prefetch depth A/B (HEAD PF=6 vs PF=8 / PF=4) and full-line staged stores (working tree)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3v
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py -k "dswiglu or fused or model_step" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; echo "pytest rc $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ab_kernels.py --alt nanodiloco_amd/_lib/alt/libnd_kernels_6f93c1d.so --what epi > $O/ab_stage.log 2>&1; rc=$?; cat $O/ab_stage.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ab_kernels.py --alt nanodiloco_amd/_lib/alt/libnd_kernels_6f93c1d_pf8.so --what epi > $O/ab8.log 2>&1; rc=$?; cat $O/ab8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ab_kernels.py --alt nanodiloco_amd/_lib/alt/libnd_kernels_6f93c1d_pf4.so --what epi > $O/ab4.log 2>&1; rc=$?; cat $O/ab4.log; exit $rc
