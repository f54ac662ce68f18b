#!/bin/bash
# attention forward 3-slot DMA ring: attention tests, then in-process A/B against the HEAD library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2attn
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attn or attention" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r2attn/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r2attn/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/ab_kernels.py --alt nanodiloco_amd/_lib/alt/${ALT} --what attn --rounds 7 > gpurun_out/r2attn/ab.log 2>&1 || exit $?
cat gpurun_out/r2attn/ab.log
if [ -n "$STEP" ]; then
timeout -k 10 300 python scripts/ab_kernels.py --alt nanodiloco_amd/_lib/alt/${ALT} --what step --rounds 5 > gpurun_out/r2attn/ab_step.log 2>&1 || exit $?
cat gpurun_out/r2attn/ab_step.log
fi
